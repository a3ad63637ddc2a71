// waves/Generator.h — drop-in for Waves::Generator / Waves::GeneratorSettings
// (reference src/Generator.h:12-93). Same members and semantics; the GLSL kernels are replaced by
// the fused HIP row/column passes of liboceanfft.
#pragma once

#include <cstddef>
#include <cstdint>
#include <type_traits>
#include <utility>

#include "oceanfft.h"
#include "vision/RenderDevice.h"
#include "waves/FFTCalculator.h"

namespace Waves
{

// glm::ivec2 stand-in with the same layout (the reference's only glm use in the settings,
// src/Generator.h:14). It converts to and from any {x, y} vector type, so reference code that
// writes `settings.seed = glm::ivec2(a, b)` (or reads it back into one) compiles unchanged.
struct IVec2
{
  int32_t x = 0, y = 0;

  constexpr IVec2() = default;
  constexpr IVec2(int32_t x_, int32_t y_) : x(x_), y(y_) {}
  template <class V, class = decltype(std::declval<const V&>().x + std::declval<const V&>().y),
            class = std::enable_if_t<!std::is_same<std::decay_t<V>, IVec2>::value>>
  constexpr IVec2(const V& v) : x(static_cast<int32_t>(v.x)), y(static_cast<int32_t>(v.y))
  {
  }
  template <class V, class = decltype(V{int32_t{}, int32_t{}})>
  constexpr explicit operator V() const
  {
    return V{x, y};
  }
  int32_t& operator[](int i) { return i == 0 ? x : y; }
  const int32_t& operator[](int i) const { return i == 0 ? x : y; }
  friend constexpr bool operator==(const IVec2& a, const IVec2& b) { return a.x == b.x && a.y == b.y; }
  friend constexpr bool operator!=(const IVec2& a, const IVec2& b) { return !(a == b); }
};
static_assert(sizeof(IVec2) == 8 && std::is_trivially_copyable<IVec2>::value, "IVec2 must match glm::ivec2");

// src/Generator.h:12-30 — identical defaults and 64-byte layout.
struct GeneratorSettings
{
  IVec2 seed = {12342, 8934};  // The seed for random generation.

  float U_10 = 40.0f;         // The speed of the wind.
  float theta_0 = 25.0f;      // The CCW direction of the wind rel. to +x-axis.
  float F = 800000.0f;        // The distance to a downwind shore (fetch).
  float g = 9.8f;             // The acceleration due to gravity.
  float swell = 0.5f;         // The factor of non-wind based waves.
  float h = 100.0f;           // The depth of the ocean.
  float displacement = 0.4f;  // The scalar used in displacing the vertices.
  float time = 0.0f;          // The time in seconds since the program began.
  float planeSize = 40.0f;    // The size of the plane in meters that this plane is simulating.
  float scale = 1.0f;         // The global heightmap scalar.
  float spread = 0.2f;        // The intensity of waves perp. to wind.
  int boundWavelength = 0;    // Whether or not we bound the wavelength (1 = bound, 0 = unbound)
  float wavelengthMin = 0.0f; // The minimum wavelength that is allowed
  float wavelengthMax = 0.0f; // The maximum wavelength that is allowed
};
static_assert(sizeof(GeneratorSettings) == 64, "GeneratorSettings must stay 64 bytes (std140 UBO)");

class Generator
{
public:
  // src/Generator.h:36-37
  Generator(Vision::RenderDevice* device, FFTCalculator* calc);
  ~Generator();
  Generator(const Generator&) = delete;
  Generator& operator=(const Generator&) = delete;

  // src/Generator.h:41. If the spectrum is modified, pass updateOcean = true to the next call.
  GeneratorSettings& GetOceanSettings();

  // src/Generator.h:45. time += timestep; (re)seed h0 if requested or first call; evolve, 2D iFFT
  // of both packed maps, Jacobian. Enqueued on the device's stream (no host sync).
  void CalculateOcean(float timestep, bool updateOcean = false);

  // src/Generator.h:48-50. heightMap = (h, dh/dx, dh/dz, Dx), displacementMap =
  // (Dz, dDx/dx, dDz/dz, dDx/dz), jacobian = R32F. IDs resolve through the RenderDevice.
  Vision::ID GetHeightMap() const { return heightMap; }
  Vision::ID GetDisplacementMap() const { return displacementMap; }
  Vision::ID GetJacobianMap() const { return jacobian; }

  // src/Generator.h:53. Kernels are compiled into liboceanfft for gfx950; nothing to reload.
  void LoadShaders(bool reload = false);

  // Extension (no reference counterpart): the C-ABI generator behind this object, for ABI calls
  // such as ocean_surface_sample_plane (waves/Surface.h).
  ocean_generator* GetHandle() const { return gen; }

private:
  Vision::RenderDevice* renderDevice = nullptr;
  FFTCalculator* fftCalc = nullptr;
  std::size_t textureSize = 0;
  ocean_generator* gen = nullptr;
  Vision::ID heightMap = 0;
  Vision::ID displacementMap = 0;
  Vision::ID jacobian = 0;
};

}  // namespace Waves
