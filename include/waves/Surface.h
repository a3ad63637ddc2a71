// waves/Surface.h — the renderer's use of the maps as a compute step.
// WaveRenderer::Render (reference src/Renderer.cpp:53-72) binds the three generators' maps and
// draws the plane mesh with resources/waveShader.glsl, whose vertex stage displaces each vertex by
// the cascades (:101-110) and whose fragment stage derives the slope normal and foam (:127-144).
// SurfaceSampler evaluates that sampling per mesh vertex on the GPU and hands the renderer final
// vertices instead of textures.
#pragma once

#include <vector>

#include "oceanfft.h"
#include "vision/RenderDevice.h"
#include "waves/Generator.h"

namespace Waves
{

class SurfaceSampler
{
public:
  explicit SurfaceSampler(Vision::RenderDevice* device) : renderDevice(device) {}
  ~SurfaceSampler();
  SurfaceSampler(const SurfaceSampler&) = delete;
  SurfaceSampler& operator=(const SurfaceSampler&) = delete;

  // The reference plane mesh (res x res quads, src/Renderer.cpp:18) around the camera
  // (camera = viewInverse[3].xyz, then forward.xz = -viewInverse[0].xz, waveShader.glsl:84-92),
  // sampled on generators[i]'s maps (Renderer.cpp:62-72). Returns a buffer texture of
  // 2*(res+1) x (res+1) RGBA32F texels: per vertex (x, y, z, jacobian), (nx, ny, nz, 0).
  // Enqueued on the device's stream; the texture is owned by the sampler and reused.
  Vision::ID Sample(const std::vector<Generator*>& generators, const float camera[5], int res);

private:
  Vision::RenderDevice* renderDevice = nullptr;
  Vision::ID vertices = 0;
  int verticesRes = 0;
};

}  // namespace Waves
