"""bench.py's multi-rank plumbing on CPU: world_size 2 over gloo (127.0.0.1). Each rank runs the same
barrier + max-over-ranks protocol the GPU bench uses; the aggregate must be whole-job throughput."""
import importlib.util
import os
import socket

import pytest
import torch.multiprocessing as mp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank))
    spec = importlib.util.spec_from_file_location("bench", os.path.join(ROOT, "bench.py"))
    b = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(b)
    r, w, _ = b.dist_setup()
    assert (r, w) == (rank, world)
    b.barrier(w)
    local_elapsed = 1.0 + rank  # rank 1 is the slow one
    el_max = b.max_over_ranks(local_elapsed, w)
    # per-rank disjoint work: cascades owned by this rank in the weak leg (8 each) ...
    owned = [(b.cascade_settings(r, c)["planeSize"],) + tuple(b.cascade_settings(r, c)["seed"]) for c in range(8)]
    # ... and in the strong-scaling headline (the job's 8 global cascades split 8 / world per rank)
    strong = [(c,) + (b.cascade_settings(0, c)["planeSize"],) + tuple(b.cascade_settings(0, c)["seed"])
              for c in b.rank_cascades(8, r, w)]
    import torch.distributed as dist

    gathered = [None] * w
    dist.all_gather_object(gathered, owned)
    gathered_strong = [None] * w
    dist.all_gather_object(gathered_strong, strong)
    b.barrier(w)
    dist.destroy_process_group()
    q.put((rank, el_max, gathered, gathered_strong))


@pytest.mark.timeout(120)
def test_world2_max_over_ranks_and_disjoint_cascades():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = [q.get(timeout=100) for _ in procs]
    for p in procs:
        p.join(timeout=30)
        assert p.exitcode == 0
    spec = importlib.util.spec_from_file_location("bench", os.path.join(ROOT, "bench.py"))
    b = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(b)
    one_gpu = [(c,) + (b.cascade_settings(0, c)["planeSize"],) + tuple(b.cascade_settings(0, c)["seed"]) for c in range(8)]
    for rank, el_max, gathered, gathered_strong in res:
        assert el_max == 2.0  # max over ranks, not rank-local time
        flat = [tuple(k) for ranks in gathered for k in ranks]
        assert len(set(flat)) == len(flat)  # no cascade computed twice across ranks
        # strong scaling: 4 cascades per rank, disjoint, together exactly the 1-GPU job's 8
        assert [len(x) for x in gathered_strong] == [4, 4]
        strong = [tuple(k) for ranks in gathered_strong for k in ranks]
        assert len(set(strong)) == 8 and sorted(strong) == sorted(one_gpu)


def _a2a_worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank))
    import torch
    import torch.distributed as dist

    dist.init_process_group("gloo")
    import sys

    sys.path.insert(0, ROOT)
    from oceansimulation_amd.slab import TorchExchange, block_moves

    nbytes = 16 * world
    ex = TorchExchange(nbytes, torch.device("cpu"))
    ex.send.copy_(torch.tensor([rank * 16 + qq for qq in range(world) for _ in range(16)], dtype=torch.uint8))
    ex()
    got = ex.recv.tolist()
    # the emulated exchange's block map must describe exactly what the collective did
    expect = [0] * nbytes
    for s, so, dst, do, size in block_moves(world, nbytes):
        if dst == rank:
            expect[do:do + size] = [s * 16 + (so // 16)] * size
    dist.destroy_process_group()
    q.put((rank, got == expect))


@pytest.mark.timeout(120)
def test_world2_alltoall_matches_emulated_block_moves():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_a2a_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = [q.get(timeout=100) for _ in procs]
    for p in procs:
        p.join(timeout=30)
        assert p.exitcode == 0
    assert all(ok for _, ok in res)


def _gather_worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank))
    import sys

    import torch.distributed as dist

    dist.init_process_group("gloo")
    sys.path.insert(0, ROOT)
    from oceansimulation_amd.slab import torch_gather_bytes

    spec = importlib.util.spec_from_file_location("bench", os.path.join(ROOT, "bench.py"))
    b = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(b)
    # what put_leg hands ocean_peers_connect: every rank's 256-byte handle, in rank order
    blob = bytes([rank]) * 256
    got = torch_gather_bytes(blob)
    # the verdicts every multi-rank leg agrees on before it branches (MIN over ranks)
    agree_all = b.ranks_agree(True, world)
    agree_one_fails = b.ranks_agree(rank != 1, world)
    dist.destroy_process_group()
    q.put((rank, [g[:1] for g in got], [len(g) for g in got], agree_all, agree_one_fails))


@pytest.mark.timeout(120)
def test_world2_peer_handles_gather_in_rank_order_and_verdicts_agree():
    """The one-sided exchange's handle exchange (slab.torch_gather_bytes, an all_gather_object) gives
    every rank all handles in rank order, and bench.ranks_agree makes every rank take the branch of the
    most pessimistic one (a rank whose connect or check failed stops all of them)."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_gather_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = [q.get(timeout=100) for _ in procs]
    for p in procs:
        p.join(timeout=30)
        assert p.exitcode == 0
    for rank, heads, lens, agree_all, agree_one_fails in res:
        assert heads == [bytes([0]), bytes([1])] and lens == [256, 256]
        assert agree_all is True and agree_one_fails is False
