// waves/SlabGenerator.h — one cascade split over P GPUs (one process per GPU), the C++ face of the
// slab C ABI and its RCCL exchange (oceanfft.h "slab decomposition" / "the slab exchange over RCCL").
// No reference counterpart: the reference runs each Waves::Generator on one device
// (src/Generator.cpp:45-83). Settings, CalculateOcean and the map getters mean what they mean on
// Waves::Generator (waves/Generator.h), the maps holding this rank's row slab (GetRows() rows of
// N texels, starting at global row GetFirstRow()).
#pragma once

#include <array>

#include "oceanfft.h"
#include "vision/RenderDevice.h"
#include "waves/FFTCalculator.h"
#include "waves/Generator.h"

namespace Waves
{

// The communicator of the P ranks of one grid (RCCL over xGMI), on the current HIP device.
class SlabComm
{
public:
  using UniqueId = std::array<unsigned char, OCEAN_COMM_ID_BYTES>;
  // ncclGetUniqueId on one rank; the caller hands it to every rank (MPI, a file, torch.distributed).
  static UniqueId NewUniqueId();
  // ncclCommInitRank: collective over the `ranks` processes.
  SlabComm(const UniqueId& id, int ranks, int rank);
  // Wraps a communicator the caller owns (an ncclComm_t); the destructor leaves it alone.
  SlabComm(void* ncclComm, int ranks, int rank);
  ~SlabComm();
  SlabComm(const SlabComm&) = delete;
  SlabComm& operator=(const SlabComm&) = delete;

  int GetRank() const { return rank; }
  int GetRanks() const { return ranks; }
  ocean_comm* GetHandle() const { return comm; }

private:
  ocean_comm* comm = nullptr;
  int ranks = 0, rank = 0;
};

class SlabGenerator
{
public:
  // This rank's slab of one calc->GetTextureResolution()^2 cascade (ranks a power of two <= 16).
  SlabGenerator(Vision::RenderDevice* device, FFTCalculator* calc, SlabComm* comm);
  ~SlabGenerator();
  SlabGenerator(const SlabGenerator&) = delete;
  SlabGenerator& operator=(const SlabGenerator&) = delete;

  // Same settings block as Waves::Generator; every rank must hold the same values.
  GeneratorSettings& GetOceanSettings();

  // One frame on the device's stream: time += timestep, h0 of this rank's columns if needed, column
  // pass, the all-to-all, row pass. Every rank calls it with the same arguments.
  void CalculateOcean(float timestep, bool updateOcean = false);
  // The same frame with the all-to-all on a second stream beside the next frame's column pass: the
  // maps lag the last call by one frame until Flush().
  void CalculateOceanPipelined(float timestep, bool updateOcean = false);
  void Flush();

  // The row slab's maps (GetRows() x N), as Waves::Generator's.
  Vision::ID GetHeightMap() const { return heightMap; }
  Vision::ID GetDisplacementMap() const { return displacementMap; }
  Vision::ID GetJacobianMap() const { return jacobian; }
  int GetFirstRow() const { return row0; }
  int GetRows() const { return rows; }
  ocean_generator* GetHandle() const { return gen; }

private:
  Vision::RenderDevice* renderDevice = nullptr;
  SlabComm* slabComm = nullptr;
  ocean_generator* gen = nullptr;
  int row0 = 0, rows = 0;
  Vision::ID heightMap = 0;
  Vision::ID displacementMap = 0;
  Vision::ID jacobian = 0;
};

}  // namespace Waves
