// Waves::SurfaceSampler over ocean_surface_sample_plane (include/oceanfft.h).
#include "waves/Surface.h"

#include <stdexcept>
#include <string>

namespace Waves
{

SurfaceSampler::~SurfaceSampler()
{
  if (vertices)
    renderDevice->DestroyTexture2D(vertices);
}

Vision::ID SurfaceSampler::Sample(const std::vector<Generator*>& generators, const float camera[5], int res)
{
  if (!vertices || verticesRes != res)
  {
    if (vertices)
      renderDevice->DestroyTexture2D(vertices);
    Vision::Texture2DDesc desc;
    desc.Width = 2 * (res + 1);
    desc.Height = res + 1;
    desc.PixelType = Vision::PixelType::RGBA32Float;
    vertices = renderDevice->CreateTexture2D(desc);
    verticesRes = res;
  }
  std::vector<ocean_generator*> gens;
  std::vector<int> cascades;
  for (auto* g : generators)
  {
    gens.push_back(g->GetHandle());
    cascades.push_back(0);
  }
  const int rc = ocean_surface_sample_plane(gens.data(), cascades.data(), (int)gens.size(), camera, res,
                                            static_cast<float*>(renderDevice->GetTexturePointer(vertices)));
  if (rc != OCEAN_OK)
    throw std::runtime_error(std::string("SurfaceSampler::Sample: ") + ocean_last_error());
  return vertices;
}

}  // namespace Waves
