// vision/RenderDevice.h — minimal HIP-backed stand-in for the slice of the Vision engine's
// RenderDevice that the reference hot path calls (call sites: src/FFTCalculator.cpp:26-113,
// src/Generator.cpp:20-154). The reference's Vision submodule (.gitmodules:1-3) is not part of
// this build; this shim gives Waves::Generator / Waves::FFTCalculator their original constructor
// signatures. A Vision::ID names an HBM buffer; "command encoding" is issuing on one HIP stream.
#pragma once

#include <hip/hip_runtime_api.h>

#include <cstddef>
#include <cstdint>
#include <unordered_map>

namespace Vision
{

using ID = uint32_t;  // 0 = none, as in the reference (src/Generator.h:61-92)

enum class PixelType
{
  RGBA32Float,  // 16 B texels (heightMap, displacementMap, spectra)
  R32Float      // 4 B texels (jacobian)
};

enum class MinMagFilter { Nearest, Linear };
enum class EdgeAddressMode { Repeat, ClampToEdge };
enum class ImageAccess { ReadOnly, WriteOnly, ReadWrite };

// Fields used by src/Generator.cpp:106-116 and src/FFTCalculator.cpp:35-44.
struct Texture2DDesc
{
  std::size_t Width = 0;
  std::size_t Height = 0;
  ::Vision::PixelType PixelType = ::Vision::PixelType::RGBA32Float;
  MinMagFilter MinFilter = MinMagFilter::Linear;
  MinMagFilter MagFilter = MinMagFilter::Linear;
  EdgeAddressMode AddressModeS = EdgeAddressMode::Repeat;
  EdgeAddressMode AddressModeT = EdgeAddressMode::Repeat;
  bool WriteOnly = false;
  const void* Data = nullptr;
};

class RenderDevice
{
public:
  // All work of objects created on this device is issued on `stream` (nullptr = default stream).
  explicit RenderDevice(hipStream_t stream = nullptr);
  ~RenderDevice();
  RenderDevice(const RenderDevice&) = delete;
  RenderDevice& operator=(const RenderDevice&) = delete;

  // Textures (device-owned HBM buffers, row-major, x fastest).
  ID CreateTexture2D(const Texture2DDesc& desc);
  void DestroyTexture2D(ID id);
  void SetTexture2DDataRaw(ID id, const void* data);  // host -> device, whole texture
  // Registers memory owned by someone else (e.g. a Generator's maps); Destroy only forgets it.
  ID RegisterTexture2D(void* device_ptr, std::size_t width, std::size_t height, PixelType type);

  // HIP-native interop (what a HIP renderer binds instead of a sampler unit).
  void* GetTexturePointer(ID id) const;
  std::size_t GetTextureWidth(ID id) const;
  std::size_t GetTextureHeight(ID id) const;
  PixelType GetTexturePixelType(ID id) const;
  void GetTexture2DDataRaw(ID id, void* host_out);  // device -> host, synchronises

  // Command encoding == stream order. Barriers are implied by stream order (the reference's
  // ImageBarrier after each dispatch, src/FFTCalculator.cpp:98-112).
  void BeginCommandBuffer() {}
  void SubmitCommandBuffer();  // waits for the stream (the reference's submit + present fence)
  void BeginComputePass() {}
  void EndComputePass() {}
  void ImageBarrier() {}

  hipStream_t GetStream() const { return stream; }

private:
  struct Texture
  {
    void* ptr = nullptr;
    std::size_t width = 0, height = 0;
    PixelType type = PixelType::RGBA32Float;
    bool owned = false;
  };
  const Texture& Get(ID id) const;

  hipStream_t stream = nullptr;
  ID nextID = 1;
  std::unordered_map<ID, Texture> textures;
};

inline std::size_t BytesPerTexel(PixelType t) { return t == PixelType::RGBA32Float ? 16 : 4; }

}  // namespace Vision
