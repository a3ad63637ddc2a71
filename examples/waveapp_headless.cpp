// waveapp_headless.cpp — the reference application's real workload without a window
// (SURVEY §8f rank 1): WaveApp's scene (reference src/Waves.cpp:14-39) driven through the C++
// drop-in exactly like WaveApp::OnUpdate (src/Waves.cpp:59-106), plus the renderer's sampling of
// the maps (waves/Surface.h) and an on-disk export of the last frame.
//
//   one FFTCalculator(N) shared by 3 Generators, plane sizes 5/17/101 m, boundWavelength = 1,
//   wavelength bounds per generator; per frame:
//     dt = 0 while "Q" is held (--freeze A:B, frames A..B-1)            src/Waves.cpp:86-87
//     CalculateOcean(dt, updateSpectrum) for every generator             src/Waves.cpp:90-91
//     the renderer's vertex displacement / normals / foam on the mesh    src/Renderer.cpp:53-84
//   settings edits (--edit F:G.field=value, applied before frame F) set updateSpectrum and redo the
//   wavelength bookkeeping of DrawUI (src/Waves.cpp:177-207). The reference never clears
//   updateSpectrum (src/Waves.cpp:93-94 is commented out), so h0 is re-seeded every frame; with
//   --reseed on-edit it is re-seeded only on the first frame and after edits (the commented-out
//   intent).
//
// Usage: waveapp_headless [--n 256] [--frames 600] [--dt 0.0166667] [--freeze A:B]...
//                         [--edit F:G.field=value]... [--reseed reference|on-edit]
//                         [--mesh RES (0 = no surface step)] [--dump DIR]
// Prints one JSON line. --dump DIR writes height_G.npy, disp_G.npy, jac_G.npy (G = 0..2),
// surface.npy ((RES+1)^2 x 8 floats) and scene.json for the last frame.
#include <hip/hip_runtime_api.h>

#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "waves/FFTCalculator.h"
#include "waves/Generator.h"
#include "waves/Surface.h"

namespace
{

struct Edit
{
  int frame = 0, gen = 0;
  std::string field;
  float value = 0.0f;
};

bool set_field(Waves::GeneratorSettings& s, const std::string& f, float v)
{
  // the fields WaveApp::DrawUI edits (src/Waves.cpp:188-198)
  if (f == "U_10") s.U_10 = v;
  else if (f == "theta_0") s.theta_0 = v;
  else if (f == "g") s.g = v;
  else if (f == "scale") s.scale = v;
  else if (f == "displacement") s.displacement = v;
  else if (f == "swell") s.swell = v;
  else if (f == "spread") s.spread = v;
  else if (f == "h") s.h = v;
  else if (f == "F") s.F = v;
  else if (f == "planeSize") s.planeSize = v;
  else return false;
  return true;
}

// numpy .npy v1.0, little-endian float32, C order
bool write_npy(const std::string& path, const float* data, const std::vector<size_t>& shape)
{
  std::string dims;
  size_t count = 1;
  for (size_t d : shape)
  {
    dims += std::to_string(d) + ",";
    count *= d;
  }
  if (shape.size() > 1)
    dims.pop_back();
  std::string header = "{'descr': '<f4', 'fortran_order': False, 'shape': (" + dims + "), }";
  const size_t total = 10 + header.size() + 1;
  header.append((64 - total % 64) % 64, ' ');
  header += '\n';
  FILE* f = std::fopen(path.c_str(), "wb");
  if (!f)
    return false;
  const unsigned char magic[8] = {0x93, 'N', 'U', 'M', 'P', 'Y', 1, 0};
  const uint16_t hl = (uint16_t)header.size();
  bool ok = std::fwrite(magic, 1, 8, f) == 8 && std::fwrite(&hl, 2, 1, f) == 1 &&
            std::fwrite(header.data(), 1, header.size(), f) == header.size() &&
            std::fwrite(data, sizeof(float), count, f) == count;
  return std::fclose(f) == 0 && ok;
}

void usage()
{
  std::fprintf(stderr, "usage: waveapp_headless [--n N] [--frames K] [--dt S] [--freeze A:B]... "
                       "[--edit F:G.field=value]... [--reseed reference|on-edit] [--mesh RES] [--dump DIR]\n");
}

}  // namespace

int main(int argc, char** argv)
{
  int n = 256, frames = 600, mesh = 1024;
  float dt = 1.0f / 60.0f;
  bool reseed_every_frame = true;
  std::string dump;
  std::vector<std::pair<int, int>> freezes;
  std::vector<Edit> edits;
  for (int i = 1; i < argc; i++)
  {
    const std::string a = argv[i];
    const char* v = i + 1 < argc ? argv[i + 1] : nullptr;
    if (!v)
    {
      usage();
      return 2;
    }
    if (a == "--n") n = std::atoi(v);
    else if (a == "--frames") frames = std::atoi(v);
    else if (a == "--dt") dt = std::strtof(v, nullptr);
    else if (a == "--mesh") mesh = std::atoi(v);
    else if (a == "--dump") dump = v;
    else if (a == "--reseed") reseed_every_frame = std::string(v) != "on-edit";
    else if (a == "--freeze")
    {
      int x = 0, y = 0;
      if (std::sscanf(v, "%d:%d", &x, &y) != 2)
      {
        usage();
        return 2;
      }
      freezes.push_back({x, y});
    }
    else if (a == "--edit")
    {
      Edit e;
      char field[64] = {0};
      if (std::sscanf(v, "%d:%d.%63[^=]=%f", &e.frame, &e.gen, field, &e.value) != 4 || e.gen < 0 || e.gen > 2)
      {
        usage();
        return 2;
      }
      e.field = field;
      edits.push_back(e);
    }
    else
    {
      usage();
      return 2;
    }
    i++;
  }

  try
  {
    Vision::RenderDevice device;
    Waves::FFTCalculator fft(&device, (std::size_t)n);
    std::vector<Waves::Generator*> generators;
    static const float primeFactors[] = {5.0f, 17.0f, 101.0f};  // src/Waves.cpp:27
    for (int i = 0; i < 3; i++)
    {
      auto* g = new Waves::Generator(&device, &fft);
      Waves::GeneratorSettings& s = g->GetOceanSettings();
      s.planeSize = primeFactors[i];
      s.boundWavelength = 1;
      s.wavelengthMax = s.planeSize / 2.0;
      s.wavelengthMin = (i == 0) ? 0.0 : primeFactors[i - 1] / 2.0;
      generators.push_back(g);
    }
    Waves::SurfaceSampler sampler(&device);
    const float camera[5] = {0.0f, 5.0f, 0.0f, -0.70711f, 0.70711f};  // src/Renderer.cpp:15-16
    bool updateSpectrum = true;  // src/Waves.h:31
    Vision::ID surface = 0;

    device.BeginCommandBuffer();
    device.SubmitCommandBuffer();
    const auto t0 = std::chrono::steady_clock::now();
    int frozen = 0, reseeds = 0;
    for (int f = 0; f < frames; f++)
    {
      bool edited = false;
      for (const Edit& e : edits)
        if (e.frame == f)
        {
          if (!set_field(generators[e.gen]->GetOceanSettings(), e.field, e.value))
          {
            std::fprintf(stderr, "unknown field %s\n", e.field.c_str());
            return 2;
          }
          edited = true;
        }
      if (edited)
      {
        updateSpectrum = true;
        for (int i = 0; i < 3; i++)  // src/Waves.cpp:199-208
        {
          Waves::GeneratorSettings& s = generators[i]->GetOceanSettings();
          s.wavelengthMax = s.planeSize / 2.0;
          s.wavelengthMin = (i == 0) ? 0.0 : generators[i - 1]->GetOceanSettings().planeSize / 2.0;
        }
      }
      float step = dt;
      for (auto& fr : freezes)
        if (f >= fr.first && f < fr.second)
          step = 0.0f;  // "Q" held: src/Waves.cpp:86-87
      frozen += step == 0.0f;
      device.BeginCommandBuffer();
      for (auto* g : generators)
        g->CalculateOcean(step, updateSpectrum);
      reseeds += updateSpectrum;
      if (!reseed_every_frame)
        updateSpectrum = false;
      if (mesh > 0)
        surface = sampler.Sample(generators, camera, mesh);
      device.SubmitCommandBuffer();
    }
    const double secs = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();

    if (!dump.empty())
    {
      const size_t texels = (size_t)n * n;
      std::vector<float> buf(texels * 4);
      for (int i = 0; i < 3; i++)
      {
        const std::string s = std::to_string(i);
        device.GetTexture2DDataRaw(generators[i]->GetHeightMap(), buf.data());
        bool ok = write_npy(dump + "/height_" + s + ".npy", buf.data(), {(size_t)n, (size_t)n, 4});
        device.GetTexture2DDataRaw(generators[i]->GetDisplacementMap(), buf.data());
        ok = ok && write_npy(dump + "/disp_" + s + ".npy", buf.data(), {(size_t)n, (size_t)n, 4});
        device.GetTexture2DDataRaw(generators[i]->GetJacobianMap(), buf.data());
        ok = ok && write_npy(dump + "/jac_" + s + ".npy", buf.data(), {(size_t)n, (size_t)n});
        if (!ok)
        {
          std::fprintf(stderr, "cannot write %s\n", dump.c_str());
          return 1;
        }
      }
      if (mesh > 0)
      {
        const size_t pts = (size_t)(mesh + 1) * (mesh + 1);
        std::vector<float> v(pts * 8);
        device.GetTexture2DDataRaw(surface, v.data());
        write_npy(dump + "/surface.npy", v.data(), {pts, 8});
      }
      FILE* js = std::fopen((dump + "/scene.json").c_str(), "w");
      if (js)
      {
        std::fprintf(js, "{\"n\": %d, \"frames\": %d, \"mesh\": %d, \"camera\": [%g, %g, %g, %g, %g], \"cascades\": [", n,
                     frames, mesh, camera[0], camera[1], camera[2], camera[3], camera[4]);
        for (int i = 0; i < 3; i++)
        {
          const Waves::GeneratorSettings& s = generators[i]->GetOceanSettings();
          std::fprintf(js, "%s{\"planeSize\": %.9g, \"time\": %.9g, \"U_10\": %.9g, \"displacement\": %.9g}",
                       i ? ", " : "", s.planeSize, s.time, s.U_10, s.displacement);
        }
        std::fprintf(js, "]}\n");
        std::fclose(js);
      }
    }
    std::printf("{\"app\": \"waveapp_headless\", \"n\": %d, \"cascades\": 3, \"frames\": %d, \"frozen_frames\": %d, "
                "\"reseeded_frames\": %d, \"reseed\": \"%s\", \"mesh_vertices\": %lld, \"seconds\": %.6f, "
                "\"ms_per_frame\": %.6f, \"frames_per_s\": %.3f, \"height_field_points_per_s\": %.6e, "
                "\"final_time\": [%.9g, %.9g, %.9g]}\n",
                n, frames, frozen, reseeds, reseed_every_frame ? "reference (every frame)" : "on-edit",
                mesh > 0 ? (long long)(mesh + 1) * (mesh + 1) : 0LL, secs, 1e3 * secs / frames, frames / secs,
                3.0 * n * n * frames / secs, generators[0]->GetOceanSettings().time,
                generators[1]->GetOceanSettings().time, generators[2]->GetOceanSettings().time);
    for (auto* g : generators)
      delete g;
  }
  catch (const std::exception& e)
  {
    std::fprintf(stderr, "waveapp_headless: %s\n", e.what());
    return 1;
  }
  return 0;
}
