"""One rank of a multi-process slab grid over the one-sided exchange (ocean_peers), for
tests/test_gpu_peers.py: every rank is its own process (here all on GPU 0), the IPC handles travel
over a gloo group, and each rank checks its row slab against a whole-grid generator in its own
process, bit for bit on the device. Prints one JSON line; exit status 0 only when everything matched.

    python tests/peer_rank.py RANK WORLD PORT N
"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import torch  # noqa: E402  (first: one HIP runtime for torch and liboceanfft.so, tests/conftest.py)
import torch.distributed as dist  # noqa: E402


def dev_equal(a: int, b: int, nbytes: int) -> bool:
    from oceansimulation_amd import hip

    x = torch.empty(nbytes, dtype=torch.uint8, device="cuda")
    y = torch.empty_like(x)
    hip.copy_d2d(x.data_ptr(), a, nbytes)
    hip.copy_d2d(y.data_ptr(), b, nbytes)
    return bool(torch.equal(x, y))


def main() -> int:
    rank, world, port, n = (int(v) for v in sys.argv[1:5])
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    import oceansimulation_amd as ocean
    from oceansimulation_amd import capi
    from oceansimulation_amd.slab import PeerExchange, SlabGenerator, torch_gather_bytes

    L = capi.lib()
    out = {"rank": rank, "world": world, "n": n}
    fft = ocean.FFTCalculator(n)
    g = SlabGenerator(fft, rank, world)
    ocean.apply_settings(g.GetOceanSettings(), planeSize=777.0)
    peers = PeerExchange(g)
    peers.set_timeout(20000)
    peers.connect(torch_gather_bytes)
    whole = ocean.Generator(fft, 1)
    ocean.apply_settings(whole.GetOceanSettings(0), planeSize=777.0)
    w = n // world

    def same() -> bool:
        fft.synchronize()
        return all(dev_equal(int(get(g.handle, 0)), int(get(whole.handle, 0)) + rank * w * n * tex, w * n * tex)
                   for get, tex in ((L.ocean_generator_height_map, 16), (L.ocean_generator_displacement_map, 16),
                                    (L.ocean_generator_jacobian_map, 4)))

    checks = {}
    for k, dt in enumerate((0.5, 1.0 / 60.0)):
        g.frame_put(peers, dt, update_ocean=(k == 0))
        whole.CalculateOcean(dt)
        peers.synchronize()
        checks[f"serial_{k}"] = same()
    steps = [0.25, 1.0 / 30.0, 0.125, 1.0 / 60.0]
    for dt in steps:
        g.frame_put_pipelined(peers, dt)
    peers.flush()
    for dt in steps:
        whole.CalculateOcean(dt)
    peers.synchronize()
    checks["pipelined"] = same()
    # a serial frame right after pipelined ones (the slots alternate on)
    g.frame_put(peers, 0.5)
    whole.CalculateOcean(0.5)
    peers.synchronize()
    checks["serial_after_pipelined"] = same()
    out["checks"] = checks
    out["ok"] = all(checks.values())
    dist.barrier()  # every rank has synchronized: no signal is in flight into anyone's flags
    peers.close()
    whole.close()
    g.close()
    fft.close()
    dist.barrier()
    dist.destroy_process_group()
    print(json.dumps(out), flush=True)
    return 0 if out["ok"] else 1


if __name__ == "__main__":
    sys.exit(main())
