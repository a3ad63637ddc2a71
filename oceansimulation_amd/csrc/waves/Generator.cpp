// Generator.cpp — Waves::Generator over the C ABI (reference src/Generator.cpp).
#include "waves/Generator.h"

#include <stdexcept>
#include <string>

namespace Waves
{

static_assert(sizeof(GeneratorSettings) == sizeof(ocean_settings), "settings layout");

Generator::Generator(Vision::RenderDevice* device, FFTCalculator* calc)
  : renderDevice(device), fftCalc(calc), textureSize(calc ? calc->GetTextureResolution() : 0)
{
  if (!device || !calc)
    throw std::runtime_error("Waves::Generator: null RenderDevice or FFTCalculator");
  if (ocean_generator_create(&gen, calc->GetPlan(), 1) != OCEAN_OK)
    throw std::runtime_error(std::string("Waves::Generator: ") + ocean_last_error());
  // The generator's HBM maps, exposed as Vision IDs (src/Generator.cpp:99-133).
  const std::size_t n = textureSize;
  heightMap = renderDevice->RegisterTexture2D(ocean_generator_height_map(gen, 0), n, n,
                                              Vision::PixelType::RGBA32Float);
  displacementMap = renderDevice->RegisterTexture2D(ocean_generator_displacement_map(gen, 0), n, n,
                                                    Vision::PixelType::RGBA32Float);
  jacobian = renderDevice->RegisterTexture2D(ocean_generator_jacobian_map(gen, 0), n, n,
                                             Vision::PixelType::R32Float);
}

Generator::~Generator()
{
  renderDevice->DestroyTexture2D(heightMap);
  renderDevice->DestroyTexture2D(displacementMap);
  renderDevice->DestroyTexture2D(jacobian);
  ocean_generator_destroy(gen);
}

GeneratorSettings& Generator::GetOceanSettings()
{
  return *reinterpret_cast<GeneratorSettings*>(ocean_generator_settings(gen, 0));
}

void Generator::CalculateOcean(float timestep, bool updateOcean)
{
  if (ocean_generator_calculate(gen, timestep, updateOcean ? 1 : 0) != OCEAN_OK)
    throw std::runtime_error(std::string("Waves::Generator::CalculateOcean: ") + ocean_last_error());
}

void Generator::LoadShaders(bool) {}

}  // namespace Waves
