// waves/SlabGenerator.h — one cascade split over P GPUs (one process per GPU), the C++ face of the
// slab C ABI and its two exchanges (oceanfft.h "slab decomposition", "the slab exchange over RCCL",
// "the one-sided slab exchange").
// No reference counterpart: the reference runs each Waves::Generator on one device
// (src/Generator.cpp:45-83). Settings, CalculateOcean and the map getters mean what they mean on
// Waves::Generator (waves/Generator.h), the maps holding this rank's row slab (GetRows() rows of
// N texels, starting at global row GetFirstRow()).
#pragma once

#include <array>
#include <vector>

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

class SlabPeers;

class SlabGenerator
{
public:
  // This rank's slab of one calc->GetTextureResolution()^2 cascade (ranks a power of two <= 16).
  SlabGenerator(Vision::RenderDevice* device, FFTCalculator* calc, SlabComm* comm);
  // The same without an RCCL communicator: frames only over the one-sided exchange (SlabPeers).
  SlabGenerator(Vision::RenderDevice* device, FFTCalculator* calc, int rank, int ranks);
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

  // The frame over the one-sided exchange (N = 8192 / 16384): the column pass stores each destination
  // block straight into the owning rank's receive slot; pipelined, the maps lag by one frame until
  // peers.Flush(). PutColumns / PutRows are its two halves, for callers that issue every rank's column
  // pass before the row passes (one process driving several ranks).
  void CalculateOceanPut(SlabPeers& peers, float timestep, bool updateOcean = false);
  void CalculateOceanPutPipelined(SlabPeers& peers, float timestep, bool updateOcean = false);
  void PutColumns(SlabPeers& peers, float timestep, bool updateOcean = false);
  void PutRows(SlabPeers& peers);

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

// This rank's end of the one-sided exchange (ocean_peers): receive slots and flag words in this GPU's
// memory, mapped by the other ranks. Connect() takes every rank's handle in rank order (the caller
// gathers them: MPI, a file, torch.distributed); ConnectLocal() joins ranks of one process.
class SlabPeers
{
public:
  using Handle = std::array<unsigned char, OCEAN_PEER_HANDLE_BYTES>;
  explicit SlabPeers(SlabGenerator& slab);
  ~SlabPeers();
  SlabPeers(const SlabPeers&) = delete;
  SlabPeers& operator=(const SlabPeers&) = delete;

  Handle GetPeerHandle() const;
  void Connect(const std::vector<Handle>& handles);
  static void ConnectLocal(const std::vector<SlabPeers*>& ranks);
  void SetTimeout(int ms);
  void SetPutCuMask(int cusPerXcd);
  void Flush();
  // Waits for this rank's streams; throws when a frame signal timed out.
  void Synchronize();
  ocean_peers* GetHandle() const { return peers; }

private:
  ocean_peers* peers = nullptr;
};

}  // namespace Waves
