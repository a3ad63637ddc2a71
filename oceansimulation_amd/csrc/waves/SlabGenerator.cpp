// SlabGenerator.cpp — Waves::SlabComm / Waves::SlabGenerator over the slab C ABI and its RCCL exchange.
#include "waves/SlabGenerator.h"

#include <stdexcept>
#include <string>

namespace Waves
{

static void check(int rc, const char* what)
{
  if (rc != OCEAN_OK)
    throw std::runtime_error(std::string(what) + ": " + ocean_last_error());
}

SlabComm::UniqueId SlabComm::NewUniqueId()
{
  UniqueId id{};
  check(ocean_comm_unique_id(id.data()), "Waves::SlabComm::NewUniqueId");
  return id;
}

SlabComm::SlabComm(const UniqueId& id, int ranks_, int rank_) : ranks(ranks_), rank(rank_)
{
  check(ocean_comm_create(&comm, id.data(), ranks, rank), "Waves::SlabComm");
}

SlabComm::SlabComm(void* ncclComm, int ranks_, int rank_) : ranks(ranks_), rank(rank_)
{
  check(ocean_comm_wrap(&comm, ncclComm, ranks, rank), "Waves::SlabComm");
}

SlabComm::~SlabComm() { ocean_comm_destroy(comm); }

SlabGenerator::SlabGenerator(Vision::RenderDevice* device, FFTCalculator* calc, SlabComm* comm)
  : SlabGenerator(device, calc, comm ? comm->GetRank() : -1, comm ? comm->GetRanks() : 0)
{
  slabComm = comm;
}

SlabGenerator::SlabGenerator(Vision::RenderDevice* device, FFTCalculator* calc, int rank, int ranks)
  : renderDevice(device)
{
  if (!device || !calc || ranks < 1)
    throw std::runtime_error("Waves::SlabGenerator: null RenderDevice, FFTCalculator or SlabComm");
  check(ocean_generator_create_slab(&gen, calc->GetPlan(), rank, ranks), "Waves::SlabGenerator");
  int r = 0, p = 0;
  if (ocean_generator_slab_info(gen, &r, &p, &row0, &rows) != OCEAN_OK)
  {
    ocean_generator_destroy(gen);
    throw std::runtime_error(std::string("Waves::SlabGenerator: ") + ocean_last_error());
  }
  const std::size_t n = calc->GetTextureResolution();
  heightMap = renderDevice->RegisterTexture2D(ocean_generator_height_map(gen, 0), n, rows,
                                              Vision::PixelType::RGBA32Float);
  displacementMap = renderDevice->RegisterTexture2D(ocean_generator_displacement_map(gen, 0), n, rows,
                                                    Vision::PixelType::RGBA32Float);
  jacobian = renderDevice->RegisterTexture2D(ocean_generator_jacobian_map(gen, 0), n, rows,
                                             Vision::PixelType::R32Float);
}

SlabGenerator::~SlabGenerator()
{
  renderDevice->DestroyTexture2D(heightMap);
  renderDevice->DestroyTexture2D(displacementMap);
  renderDevice->DestroyTexture2D(jacobian);
  ocean_generator_destroy(gen);
}

GeneratorSettings& SlabGenerator::GetOceanSettings()
{
  return *reinterpret_cast<GeneratorSettings*>(ocean_generator_settings(gen, 0));
}

void SlabGenerator::CalculateOcean(float timestep, bool updateOcean)
{
  if (!slabComm)
    throw std::runtime_error("Waves::SlabGenerator::CalculateOcean: no SlabComm (use CalculateOceanPut)");
  check(ocean_generator_slab_frame(gen, slabComm->GetHandle(), timestep, updateOcean ? 1 : 0),
        "Waves::SlabGenerator::CalculateOcean");
}

void SlabGenerator::CalculateOceanPipelined(float timestep, bool updateOcean)
{
  if (!slabComm)
    throw std::runtime_error("Waves::SlabGenerator::CalculateOceanPipelined: no SlabComm");
  check(ocean_generator_slab_frame_pipelined(gen, slabComm->GetHandle(), timestep, updateOcean ? 1 : 0),
        "Waves::SlabGenerator::CalculateOceanPipelined");
}

void SlabGenerator::Flush() { check(ocean_generator_slab_flush(gen), "Waves::SlabGenerator::Flush"); }

void SlabGenerator::CalculateOceanPut(SlabPeers& peers, float timestep, bool updateOcean)
{
  check(ocean_generator_slab_frame_put(gen, peers.GetHandle(), timestep, updateOcean ? 1 : 0),
        "Waves::SlabGenerator::CalculateOceanPut");
}

void SlabGenerator::CalculateOceanPutPipelined(SlabPeers& peers, float timestep, bool updateOcean)
{
  check(ocean_generator_slab_frame_put_pipelined(gen, peers.GetHandle(), timestep, updateOcean ? 1 : 0),
        "Waves::SlabGenerator::CalculateOceanPutPipelined");
}

void SlabGenerator::PutColumns(SlabPeers& peers, float timestep, bool updateOcean)
{
  check(ocean_generator_slab_put_columns(gen, peers.GetHandle(), timestep, updateOcean ? 1 : 0),
        "Waves::SlabGenerator::PutColumns");
}

void SlabGenerator::PutRows(SlabPeers& peers)
{
  check(ocean_generator_slab_put_rows(gen, peers.GetHandle()), "Waves::SlabGenerator::PutRows");
}

SlabPeers::SlabPeers(SlabGenerator& slab) { check(ocean_peers_create(&peers, slab.GetHandle()), "Waves::SlabPeers"); }

SlabPeers::~SlabPeers() { ocean_peers_destroy(peers); }

SlabPeers::Handle SlabPeers::GetPeerHandle() const
{
  Handle h{};
  check(ocean_peers_handle(peers, h.data()), "Waves::SlabPeers::GetPeerHandle");
  return h;
}

void SlabPeers::Connect(const std::vector<Handle>& handles)
{
  std::vector<unsigned char> all;
  for (const auto& h : handles)
    all.insert(all.end(), h.begin(), h.end());
  check(ocean_peers_connect(peers, all.data()), "Waves::SlabPeers::Connect");
}

void SlabPeers::ConnectLocal(const std::vector<SlabPeers*>& ranks)
{
  std::vector<ocean_peers*> all;
  for (auto* p : ranks)
    all.push_back(p->peers);
  check(ocean_peers_connect_local(all.data(), (int)all.size()), "Waves::SlabPeers::ConnectLocal");
}

void SlabPeers::SetTimeout(int ms) { check(ocean_peers_set_timeout(peers, ms), "Waves::SlabPeers::SetTimeout"); }

void SlabPeers::SetPutCuMask(int cusPerXcd)
{
  check(ocean_peers_set_put_cu_mask(peers, cusPerXcd), "Waves::SlabPeers::SetPutCuMask");
}

void SlabPeers::Flush() { check(ocean_peers_flush(peers), "Waves::SlabPeers::Flush"); }

void SlabPeers::Synchronize() { check(ocean_peers_synchronize(peers), "Waves::SlabPeers::Synchronize"); }

}  // namespace Waves
