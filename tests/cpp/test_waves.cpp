// test_waves.cpp — drives the C++ drop-in API the way the reference app does and checks it
// against the CPU oracle (test infrastructure: links oracle/build/liboceanoracle.so as checker).
//
// Scene = WaveApp's (src/Waves.cpp:14-39): one FFTCalculator shared by 3 Generators, plane sizes
// 5/17/101 m, boundWavelength = 1, wavelength bounds; per frame CalculateOcean(dt, true) for
// every generator (src/Waves.cpp:90-91: updateSpectrum is never cleared). Also checks
// FFTCalculator::EncodeIFFT on a random image, and Waves::SlabGenerator at world size 1 (the RCCL
// exchange with one rank, pipelined and not) against a whole-grid Waves::Generator, bit for bit, and
// two Waves::SlabGenerator ranks of one process over the one-sided exchange (Waves::SlabPeers joined
// locally), serial and pipelined, against the whole grid, bit for bit.
// Usage: test_waves [n] [frames] [slab n, 0 = skip] [put n, 0 = skip]. Exit code 0 = all within tolerance.
#include <hip/hip_runtime_api.h>

#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <random>
#include <vector>

#include "ocean_oracle.h"
#include "waves/FFTCalculator.h"
#include "waves/Generator.h"
#include "waves/SlabGenerator.h"

static double rel_err(const std::vector<float>& got, const std::vector<float>& ref, int stride, int ch)
{
  double maxref = 0, maxerr = 0;
  for (size_t i = ch; i < ref.size(); i += stride)
  {
    maxref = std::fmax(maxref, std::fabs((double)ref[i]));
    maxerr = std::fmax(maxerr, std::fabs((double)got[i] - (double)ref[i]));
  }
  return maxref > 0 ? maxerr / maxref : maxerr;
}

// Waves::SlabGenerator over a one-rank communicator (the library's RCCL all-to-all, pipelined and
// not) against Waves::Generator on the whole grid: the same kernels on the same columns, so the maps
// must agree bit for bit.
static int slab_world1(Vision::RenderDevice& device, int n, int frames)
{
  int failures = 0;
  Waves::FFTCalculator fft(&device, n);
  Waves::SlabComm comm(Waves::SlabComm::NewUniqueId(), 1, 0);
  Waves::Generator whole(&device, &fft);
  Waves::SlabGenerator serial(&device, &fft, &comm), piped(&device, &fft, &comm);
  if (serial.GetFirstRow() != 0 || serial.GetRows() != n)
  {
    std::printf("slab n=%d: row slab %d + %d, expected 0 + %d\n", n, serial.GetFirstRow(), serial.GetRows(), n);
    return 1;
  }
  for (auto* s : {&serial.GetOceanSettings(), &piped.GetOceanSettings()})
    *s = whole.GetOceanSettings();
  const float dt = 1.0f / 60.0f;
  for (int f = 0; f < frames; f++)
  {
    whole.CalculateOcean(dt, f == 0);
    serial.CalculateOcean(dt, f == 0);
    piped.CalculateOceanPipelined(dt, f == 0);
  }
  piped.Flush();
  const size_t texels = (size_t)n * n;
  std::vector<float> a(texels * 4), b(texels * 4), c(texels * 4);
  const Vision::ID ids[3][3] = {{whole.GetHeightMap(), serial.GetHeightMap(), piped.GetHeightMap()},
                                {whole.GetDisplacementMap(), serial.GetDisplacementMap(), piped.GetDisplacementMap()},
                                {whole.GetJacobianMap(), serial.GetJacobianMap(), piped.GetJacobianMap()}};
  static const char* names[3] = {"heightMap", "displacementMap", "jacobian"};
  for (int m = 0; m < 3; m++)
  {
    const size_t bytes = texels * (m == 2 ? 4 : 16);
    device.GetTexture2DDataRaw(ids[m][0], a.data());
    device.GetTexture2DDataRaw(ids[m][1], b.data());
    device.GetTexture2DDataRaw(ids[m][2], c.data());
    const bool ok_s = std::memcmp(a.data(), b.data(), bytes) == 0, ok_p = std::memcmp(a.data(), c.data(), bytes) == 0;
    std::printf("slab n=%d world 1 %s: serial %s, pipelined %s\n", n, names[m], ok_s ? "bit-exact" : "DIFFERS",
                ok_p ? "bit-exact" : "DIFFERS");
    failures += !ok_s + !ok_p;
  }
  if (serial.GetOceanSettings().time != whole.GetOceanSettings().time)
    failures++;
  return failures;
}

// Two ranks of one n x n grid in this process over the one-sided exchange: PutColumns of both ranks,
// then PutRows of both (serial frames), then pipelined frames + Flush, each rank's row slab against the
// whole grid bit for bit.
static int slab_put_two_ranks(Vision::RenderDevice& device, int n, int frames)
{
  int failures = 0;
  Waves::FFTCalculator fft(&device, n);
  Waves::Generator whole(&device, &fft);
  Waves::SlabGenerator r0(&device, &fft, 0, 2), r1(&device, &fft, 1, 2);
  Waves::SlabPeers p0(r0), p1(r1);
  Waves::SlabPeers::ConnectLocal({&p0, &p1});
  const float dt = 1.0f / 60.0f;
  auto check_rows = [&](const char* what) {
    p0.Synchronize();
    p1.Synchronize();
    const size_t half = (size_t)n * n / 2;
    std::vector<float> w(half * 2 * 4), s(half * 4);
    const Vision::ID ids[3][3] = {{whole.GetHeightMap(), r0.GetHeightMap(), r1.GetHeightMap()},
                                  {whole.GetDisplacementMap(), r0.GetDisplacementMap(), r1.GetDisplacementMap()},
                                  {whole.GetJacobianMap(), r0.GetJacobianMap(), r1.GetJacobianMap()}};
    for (int m = 0; m < 3; m++)
    {
      const size_t ch = m == 2 ? 1 : 4;
      device.GetTexture2DDataRaw(ids[m][0], w.data());
      for (int r = 0; r < 2; r++)
      {
        device.GetTexture2DDataRaw(ids[m][1 + r], s.data());
        const bool ok = std::memcmp(s.data(), w.data() + r * half * ch, half * ch * sizeof(float)) == 0;
        std::printf("one-sided n=%d %s map %d rank %d: %s\n", n, what, m, r, ok ? "bit-exact" : "DIFFERS");
        failures += !ok;
      }
    }
  };
  for (int f = 0; f < frames; f++)
  {
    whole.CalculateOcean(dt, f == 0);
    r0.PutColumns(p0, dt, f == 0);
    r1.PutColumns(p1, dt, f == 0);
    r0.PutRows(p0);
    r1.PutRows(p1);
  }
  check_rows("serial");
  for (int f = 0; f < frames; f++)
  {
    whole.CalculateOcean(dt);
    r0.CalculateOceanPutPipelined(p0, dt);
    r1.CalculateOceanPutPipelined(p1, dt);
  }
  p0.Flush();
  p1.Flush();
  check_rows("pipelined");
  return failures;
}

int main(int argc, char** argv)
{
  const int n = argc > 1 ? std::atoi(argv[1]) : 256;
  const int frames = argc > 2 ? std::atoi(argv[2]) : 3;
  const int slab_n = argc > 3 ? std::atoi(argv[3]) : 1024;
  const int put_n = argc > 4 ? std::atoi(argv[4]) : 8192;
  int failures = 0;

  Vision::RenderDevice device;  // default stream
  Waves::FFTCalculator fft(&device, n);

  // ---- EncodeIFFT on a random image (tolerance 1e-5 of max|ref| per channel) ----
  {
    Vision::Texture2DDesc desc;
    desc.Width = n;
    desc.Height = n;
    std::vector<float> img((size_t)n * n * 4), work(img.size()), out(img.size());
    std::mt19937 rng(1234);
    std::normal_distribution<float> nd(0.0f, 1.0f);
    for (auto& v : img)
      v = nd(rng);
    desc.Data = img.data();
    Vision::ID id = device.CreateTexture2D(desc);
    device.BeginCommandBuffer();
    fft.EncodeIFFT(id);
    device.SubmitCommandBuffer();
    device.GetTexture2DDataRaw(id, out.data());
    oracle_encode_ifft(n, img.data(), work.data());
    for (int ch = 0; ch < 4; ch++)
    {
      double e = rel_err(out, img, 4, ch);
      std::printf("encode_ifft n=%d ch=%d rel_err=%.3e\n", n, ch, e);
      if (!(e <= 1e-5))
        failures++;
    }
    device.DestroyTexture2D(id);
  }

  // ---- 3-cascade scene (src/Waves.cpp:20-39) ----
  std::vector<Waves::Generator*> generators;
  std::vector<oracle_settings> osettings(3);
  static const float primeFactors[] = {5.0f, 17.0f, 101.0f};
  for (int i = 0; i < 3; i++)
  {
    auto* g = new Waves::Generator(&device, &fft);
    Waves::GeneratorSettings& s = g->GetOceanSettings();
    s.planeSize = primeFactors[i];
    s.boundWavelength = 1;
    s.wavelengthMax = s.planeSize / 2.0;
    s.wavelengthMin = (i == 0) ? 0.0 : primeFactors[i - 1] / 2.0;
    static_assert(sizeof(oracle_settings) == sizeof(Waves::GeneratorSettings), "layout");
    std::memcpy(&osettings[i], &s, sizeof(s));
    generators.push_back(g);
  }

  const size_t texels = (size_t)n * n;
  std::vector<float> h0(texels * 4), height(texels * 4), disp(texels * 4), jac(texels), work(texels * 4);
  std::vector<std::vector<float>> ref_h(3), ref_d(3), ref_j(3);
  const float dt = 1.0f / 60.0f;
  for (int f = 0; f < frames; f++)
  {
    device.BeginCommandBuffer();
    for (auto* g : generators)
      g->CalculateOcean(dt, true);
    device.SubmitCommandBuffer();
  }
  for (int i = 0; i < 3; i++)
  {
    for (int f = 0; f < frames; f++)
      oracle_calculate_ocean(&osettings[i], n, dt, 1, h0.data(), height.data(), disp.data(), jac.data(),
                             work.data());
    std::vector<float> gh(texels * 4), gd(texels * 4), gj(texels);
    device.GetTexture2DDataRaw(generators[i]->GetHeightMap(), gh.data());
    device.GetTexture2DDataRaw(generators[i]->GetDisplacementMap(), gd.data());
    device.GetTexture2DDataRaw(generators[i]->GetJacobianMap(), gj.data());
    const float t_gpu = generators[i]->GetOceanSettings().time;
    if (t_gpu != osettings[i].time)
    {
      std::printf("cascade %d: time mismatch %.9g vs %.9g\n", i, t_gpu, osettings[i].time);
      failures++;
    }
    for (int ch = 0; ch < 4; ch++)
    {
      double eh = rel_err(gh, height, 4, ch), ed = rel_err(gd, disp, 4, ch);
      std::printf("cascade %d L=%g heightMap ch%d rel_err=%.3e  displacementMap ch%d rel_err=%.3e\n", i,
                  primeFactors[i], ch, eh, ch, ed);
      if (!(eh <= 1e-4) || !(ed <= 1e-4))
        failures++;
    }
    double ej = rel_err(gj, jac, 1, 0);
    std::printf("cascade %d jacobian rel_err=%.3e\n", i, ej);
    if (!(ej <= 1e-4))
      failures++;
  }
  for (auto* g : generators)
    delete g;
  if (slab_n > 0)
    failures += slab_world1(device, slab_n, frames);
  if (put_n > 0)
    failures += slab_put_two_ranks(device, put_n, frames);
  std::printf("%s (%d failures)\n", failures ? "FAIL" : "PASS", failures);
  return failures ? 1 : 0;
}
