// waves/FFTCalculator.h — drop-in for Waves::FFTCalculator (reference src/FFTCalculator.h:11-59).
// Same public surface; the radix-2 GLSL pass table and work image are replaced by the HIP
// Stockham iFFT in liboceanfft (include/oceanfft.h).
#pragma once

#include <cstddef>

#include "oceanfft.h"
#include "vision/RenderDevice.h"

namespace Waves
{

class FFTCalculator
{
public:
  // src/FFTCalculator.h:15. textureSize must be a power of two in [16, 16384] (the reference
  // silently required textureSize == 256 == fft.compute's SIZE; here other sizes work and
  // invalid ones throw std::runtime_error).
  FFTCalculator(Vision::RenderDevice* device, std::size_t textureSize = 512);
  ~FFTCalculator();
  FFTCalculator(const FFTCalculator&) = delete;
  FFTCalculator& operator=(const FFTCalculator&) = delete;

  // src/FFTCalculator.h:20-22. In-place inverse FFT of an RGBA32F textureSize^2 image
  // (N^2 * ifft2(ifftshift(.)) on xy and zw). Enqueued on the device's stream.
  void EncodeIFFT(Vision::ID image);

  std::size_t GetTextureResolution() const { return textureSize; }

  // Extension: the C-ABI plan (for batching through ocean_generator_create / ocean_fft_*).
  ocean_fft* GetPlan() const { return plan; }
  Vision::RenderDevice* GetDevice() const { return device; }

private:
  Vision::RenderDevice* device;
  std::size_t textureSize = 0;
  ocean_fft* plan = nullptr;
};

}  // namespace Waves
