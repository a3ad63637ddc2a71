// FFTCalculator.cpp — Waves::FFTCalculator over the C ABI (reference src/FFTCalculator.cpp).
#include "waves/FFTCalculator.h"

#include <stdexcept>
#include <string>

namespace Waves
{

FFTCalculator::FFTCalculator(Vision::RenderDevice* renderDevice, std::size_t size)
  : device(renderDevice), textureSize(size)
{
  if (!device)
    throw std::runtime_error("Waves::FFTCalculator: null RenderDevice");
  if (ocean_fft_create(&plan, size, device->GetStream()) != OCEAN_OK)
    throw std::runtime_error(std::string("Waves::FFTCalculator: ") + ocean_last_error());
}

FFTCalculator::~FFTCalculator() { ocean_fft_destroy(plan); }

void FFTCalculator::EncodeIFFT(Vision::ID image)
{
  if (device->GetTextureWidth(image) != textureSize || device->GetTextureHeight(image) != textureSize ||
      device->GetTexturePixelType(image) != Vision::PixelType::RGBA32Float)
    throw std::runtime_error("Waves::FFTCalculator::EncodeIFFT: image must be RGBA32F textureSize^2");
  if (ocean_fft_encode_ifft(plan, static_cast<float*>(device->GetTexturePointer(image))) != OCEAN_OK)
    throw std::runtime_error(std::string("Waves::FFTCalculator::EncodeIFFT: ") + ocean_last_error());
}

}  // namespace Waves
