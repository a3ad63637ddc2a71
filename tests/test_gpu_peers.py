"""The one-sided slab exchange (ocean_peers, include/oceanfft.h): the four-step column pass stores each
destination block straight into the owning rank's receive slot, and per-frame flag words replace the
all-to-all (the reference's CalculateOcean, src/Generator.cpp:45-83, split over ranks).

- P ranks in one process (ocean_peers_connect_local: the peers are the other ranks' buffers): serial
  frames, frames issued column-passes-first, and pipelined frames against the whole-grid generator,
  bit for bit on the device.
- Two ranks as two processes on GPU 0 (IPC handles over gloo, tests/peer_rank.py): the
  cross-process path itself, each rank checking its row slab against a whole grid.
- A rank whose peer never signals: the bounded wait gives up, and ocean_peers_synchronize reports
  OCEAN_ERR_TIMEOUT instead of hanging.
"""
import json
import os
import socket
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.fixture(scope="module")
def ocean():
    import oceansimulation_amd as o
    from oceansimulation_amd import capi

    assert capi.lib().ocean_device_count() > 0, "no GPU visible to liboceanfft.so"
    return o


def _dev_equal(ptr_a: int, ptr_b: int, nbytes: int) -> bool:
    import torch

    from oceansimulation_amd import hip

    a = torch.empty(nbytes, dtype=torch.uint8, device="cuda")
    b = torch.empty_like(a)
    hip.copy_d2d(a.data_ptr(), ptr_a, nbytes)
    hip.copy_d2d(b.data_ptr(), ptr_b, nbytes)
    return bool(torch.equal(a, b))


def _same(L, slabs, whole, n):
    from oceansimulation_amd import hip

    hip.synchronize()
    P = len(slabs)
    w = n // P
    for r, g in enumerate(slabs):
        for get, tex in ((L.ocean_generator_height_map, 16), (L.ocean_generator_displacement_map, 16),
                         (L.ocean_generator_jacobian_map, 4)):
            if not _dev_equal(int(get(g.handle, 0)), int(get(whole.handle, 0)) + r * w * n * tex, w * n * tex):
                return f"rank {r} {get.__name__}"
    return None


@pytest.mark.parametrize("n,P,four_step", [(8192, 1, True), (8192, 2, True), (8192, 8, True), (16384, 8, True),
                                           (1024, 4, True), (4096, 8, True), (8192, 4, False)])
def test_put_exchange_in_one_process_bit_exact(ocean, n, P, four_step):
    """P slab ranks over one grid, joined locally: frames issued as every rank's column pass + put
    then every rank's row pass, then pipelined frames (rank r's frame f column pass on its put stream
    beside its frame f - 1 row pass), equal the whole grid bit for bit after every check. 8192 / 16384:
    the four-step slabs (step 2 puts); 1024 / 4096 and 8192 with the four-step pass off: the strip-dealt
    slabs (the column pass puts its strips' blocks itself)."""
    from oceansimulation_amd import capi
    from oceansimulation_amd.slab import PeerExchange, SlabGenerator, emulate_put_frame

    L = capi.lib()
    fft = ocean.FFTCalculator(n)
    whole = ocean.Generator(fft, 1)
    ocean.apply_settings(whole.GetOceanSettings(0), planeSize=777.0)
    slabs = [SlabGenerator(fft, r, P) for r in range(P)]
    for g in slabs:
        ocean.apply_settings(g.GetOceanSettings(), planeSize=777.0)
    if not four_step:
        whole.set_four_step(False)
        for g in slabs:
            g.set_four_step(False)
    peers = [PeerExchange(g) for g in slabs]
    for p in peers:
        p.set_timeout(10000)
    PeerExchange.connect_local(peers)
    for k, dt in enumerate((0.5, 1.0 / 60.0, 2.0)):
        emulate_put_frame(slabs, peers, dt, update_ocean=(k == 0))
        whole.CalculateOcean(dt)
        assert _same(L, slabs, whole, n) is None, (n, P, "serial", k, _same(L, slabs, whole, n))
    steps = [0.25, 1.0 / 30.0, 0.125]
    for dt in steps:
        for g, p in zip(slabs, peers):
            g.frame_put_pipelined(p, dt)
    for p in peers:
        p.flush()
    for dt in steps:
        whole.CalculateOcean(dt)
    assert _same(L, slabs, whole, n) is None, (n, P, "pipelined")
    # the peers' own streams CU-masked (the put on 8 CUs of every XCD, step 1 and rows on the rest)
    for p in peers:
        p.set_put_cu_mask(8)
    for dt in steps:
        for g, p in zip(slabs, peers):
            g.frame_put_pipelined(p, dt)
    for p in peers:
        p.flush()
    for dt in steps:
        whole.CalculateOcean(dt)
    assert _same(L, slabs, whole, n) is None, (n, P, "pipelined, CU-masked put")
    if n == 16384:
        # the caller's streams, the row stream declared to have 64 CUs (a resident row-pass grid of 64)
        import torch

        sts = [torch.cuda.Stream() for _ in range(3)]
        for p in peers:
            p.set_streams(*(st.cuda_stream for st in sts))
            p.set_row_cus(64)
        for dt in steps:
            for g, p in zip(slabs, peers):
                g.frame_put_pipelined(p, dt)
        for p in peers:
            p.flush()
        for dt in steps:
            whole.CalculateOcean(dt)
        assert _same(L, slabs, whole, n) is None, (n, P, "pipelined, caller streams, 64 row CUs")
        for p in peers:
            p.synchronize()
            p.set_streams(None, None, None)
    for p in peers:
        p.synchronize()
        p.close()
    for g in slabs:
        g.close()
    whole.close()
    fft.close()


@pytest.mark.parametrize("n,P", [(8192, 2), (4096, 2)])
def test_put_pipelined_reseeds_stream_changes_and_close_bit_exact(ocean, n, P):
    """Stream-ordering cases of ADVICE r05, each bit-exact against the whole grid (re-seeded with the
    seeding kernel, GenerateSpectrum, as the slabs are):
    - pipelined put frames that re-seed h0 on every frame (the h0 memo off, so every re-seed writes
      h0 on the generator's stream while the previous frame's step 1 / put may still read it on the
      peers' streams), with a settings edit mid-run;
    - the same after the put CU mask changes (the peers' streams destroyed and recreated) and on the
      caller's streams (ocean_peers_set_streams), where the column pass must wait both for the last
      column pass and for the h0 writes;
    - after the peers are closed: device-copy frames whose column pass runs on the generator's
      stream after the last one ran on a destroyed stream.
    8192: the four-step slabs (step 1 and the put on two streams); 4096: the strip-dealt slabs."""
    import torch

    from oceansimulation_amd import capi
    from oceansimulation_amd.hip import DeviceBuffer
    from oceansimulation_amd.slab import PeerExchange, SlabGenerator, emulate_frame

    L = capi.lib()
    fft = ocean.FFTCalculator(n)
    whole = ocean.Generator(fft, 1)
    slabs = [SlabGenerator(fft, r, P) for r in range(P)]
    for s in [whole.GetOceanSettings(0)] + [g.GetOceanSettings() for g in slabs]:
        ocean.apply_settings(s, planeSize=777.0)
    for g in slabs:
        assert L.ocean_generator_set_h0_memo(g.handle, 0) == capi.OCEAN_OK
    peers = [PeerExchange(g) for g in slabs]
    for p in peers:
        p.set_timeout(10000)
    PeerExchange.connect_local(peers)

    def edit(**kw):
        for s in [whole.GetOceanSettings(0)] + [g.GetOceanSettings() for g in slabs]:
            ocean.apply_settings(s, **kw)

    def run(tag, steps, edits):
        for k, dt in enumerate(steps):
            if k in edits:
                edit(**edits[k])
            for g, p in zip(slabs, peers):
                g.frame_put_pipelined(p, dt, True)
            whole.GenerateSpectrum()
            whole.CalculateOcean(dt)
        for p in peers:
            p.flush()
        assert _same(L, slabs, whole, n) is None, (n, P, tag, _same(L, slabs, whole, n))

    steps = [0.25, 1.0 / 30.0, 0.125, 0.5]
    run("pipelined re-seeds", steps, {2: dict(U_10=31.0)})
    for p in peers:
        p.set_put_cu_mask(8)
    run("re-seeds after a CU-mask change", steps, {1: dict(spread=0.4)})
    sts = [torch.cuda.Stream() for _ in range(3)]
    for p in peers:
        p.set_streams(*(st.cuda_stream for st in sts))
    run("re-seeds on the caller's streams", steps, {3: dict(swell=0.7)})
    for p in peers:
        p.synchronize()
        p.set_streams(None, None, None)
        p.close()
    sends = [DeviceBuffer(g.exchange_bytes) for g in slabs]
    recvs = [DeviceBuffer(g.exchange_bytes) for g in slabs]
    edit(U_10=36.0)
    for k, dt in enumerate((0.25, 1.0 / 60.0)):
        emulate_frame(slabs, sends, recvs, dt, update_ocean=(k == 0))
        if k == 0:
            whole.GenerateSpectrum()
        whole.CalculateOcean(dt)
    assert _same(L, slabs, whole, n) is None, (n, P, "device-copy frames after close", _same(L, slabs, whole, n))
    for g in slabs:
        g.close()
    whole.close()
    fft.close()


@pytest.mark.parametrize("n,P", [(1024, 2), (8192, 2)])
def test_put_consumer_never_reads_stale_l2_lines(ocean, n, P):
    """The consumer side of the one-sided exchange's memory ordering (DESIGN.md §6 "Visibility"): frame f's
    blocks land in the slot frame f - 2's row pass read. Here every rank's slot is read into the L2s of
    all XCDs (ocean_debug_copy, three grid shapes so each XCD's L2 holds its own share of the lines,
    default-policy loads) just before the put that rewrites it; the stale copies differ from the new
    blocks (another frame time). The row pass must still see the new blocks: its kernel-start acquire,
    after the wait kernel observed every rank's ready word, drops every XCD's clean copies. Serial frames
    on the generators' stream and pipelined frames on the caller's streams (the reads on the put stream
    between frames), bit-exact against the whole grid. 1024: strip-dealt slabs, slots of ~21 MB (they fit
    the 32 MB of L2); 8192: four-step slabs."""
    import torch

    from oceansimulation_amd import capi
    from oceansimulation_amd.hip import DeviceBuffer
    from oceansimulation_amd.slab import PeerExchange, SlabGenerator
    from oceansimulation_amd.waves import debug_copy

    L = capi.lib()
    fft = ocean.FFTCalculator(n)
    whole = ocean.Generator(fft, 1)
    slabs = [SlabGenerator(fft, r, P) for r in range(P)]
    for s in [whole.GetOceanSettings(0)] + [g.GetOceanSettings() for g in slabs]:
        ocean.apply_settings(s, planeSize=61.0)
    peers = [PeerExchange(g) for g in slabs]
    for p in peers:
        p.set_timeout(10000)
    PeerExchange.connect_local(peers)
    nbytes = peers[0].debug_slot(0)[1]
    sink = DeviceBuffer(nbytes)

    def touch(slot, stream=None):
        for p in peers:
            ptr, nb = p.debug_slot(slot)
            for wgs in (1024, 1000, 1048):
                debug_copy(sink.ptr, ptr, nb, wgs, stream)

    steps = [0.5, 1.0 / 60.0, 0.25, 1.0 / 30.0, 0.125]
    for k, dt in enumerate(steps):  # serial: frame k lands in slot k % 2
        touch(k % 2)
        for g, p in zip(slabs, peers):
            g.put_columns(p, dt, k == 0)
        for g, p in zip(slabs, peers):
            g.put_rows(p)
        whole.CalculateOcean(dt)
        assert _same(L, slabs, whole, n) is None, (n, P, "serial", k, _same(L, slabs, whole, n))
    sts = [torch.cuda.Stream() for _ in range(3)]
    for p in peers:
        p.set_streams(*(st.cuda_stream for st in sts))
    f0 = len(steps)
    for k, dt in enumerate(steps):  # pipelined: frame f0 + k's put follows the reads on the put stream
        touch((f0 + k) % 2, sts[1].cuda_stream)
        for g, p in zip(slabs, peers):
            g.frame_put_pipelined(p, dt)
        whole.CalculateOcean(dt)
    for p in peers:
        p.flush()
    assert _same(L, slabs, whole, n) is None, (n, P, "pipelined", _same(L, slabs, whole, n))
    for p in peers:
        p.synchronize()
        p.set_streams(None, None, None)
        p.close()
    for g in slabs:
        g.close()
    whole.close()
    fft.close()


def test_put_timeout_is_sticky_until_recreated(ocean):
    """After a timed-out wait, ocean_peers_synchronize reports OCEAN_ERR_TIMEOUT once, clears the
    device error word, and the peers refuse every further frame (the ranks' flag counts no longer
    agree) instead of issuing frames whose waits return at once; new peers on the same generators work."""
    from oceansimulation_amd import capi
    from oceansimulation_amd.capi import OceanError
    from oceansimulation_amd.slab import PeerExchange, SlabGenerator

    L = capi.lib()
    n = 8192
    fft = ocean.FFTCalculator(n)
    whole = ocean.Generator(fft, 1)
    slabs = [SlabGenerator(fft, r, 2) for r in range(2)]
    peers = [PeerExchange(g) for g in slabs]
    PeerExchange.connect_local(peers)
    peers[0].set_timeout(300)
    slabs[0].put_columns(peers[0], 0.5, True)
    slabs[0].put_rows(peers[0])
    with pytest.raises(OceanError) as exc:
        peers[0].synchronize()
    assert exc.value.code == capi.OCEAN_ERR_TIMEOUT
    with pytest.raises(OceanError) as exc:
        slabs[0].frame_put(peers[0], 0.5)
    assert exc.value.code == capi.OCEAN_ERR_TIMEOUT and "recreate" in str(exc.value)
    with pytest.raises(OceanError):
        peers[0].synchronize()
    peers[1].synchronize()
    for p in peers:
        p.close()
    # fresh peers: both ranks' frames land, bit-exact against the whole grid at the same time
    peers = [PeerExchange(g) for g in slabs]
    for p in peers:
        p.set_timeout(10000)
    PeerExchange.connect_local(peers)
    for st in [whole.GetOceanSettings(0)] + [g.GetOceanSettings() for g in slabs]:
        st.time = 0.0  # rank 0 advanced alone above
    from oceansimulation_amd.slab import emulate_put_frame

    emulate_put_frame(slabs, peers, 0.25, True)
    whole.CalculateOcean(0.25)
    for p in peers:
        p.synchronize()
    assert _same(L, slabs, whole, n) is None
    for p in peers:
        p.close()
    for g in slabs:
        g.close()
    whole.close()
    fft.close()


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


@pytest.mark.timeout(300)
@pytest.mark.parametrize("n", [8192, 1024])
def test_put_exchange_two_processes_bit_exact(ocean, n):
    """Two slab ranks of one grid as two processes on GPU 0 (8192: four-step slabs; 1024: strip-dealt):
    the receive slots and flag words are mapped across the processes with hipIpcOpenMemHandle (the
    mapping the 8-GPU node uses over xGMI), serial and pipelined frames, each rank's row slab bit-exact
    against a whole grid."""
    port = _free_port()
    env = dict(os.environ, PYTHONUNBUFFERED="1")
    procs = [subprocess.Popen([sys.executable, os.path.join(ROOT, "tests", "peer_rank.py"), str(r), "2", str(port),
                               str(n)], stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True, env=env)
             for r in range(2)]
    results = []
    for p in procs:
        try:
            out, err = p.communicate(timeout=240)
        except subprocess.TimeoutExpired:
            for q in procs:
                q.kill()
            raise
        lines = [ln for ln in out.splitlines() if ln.startswith("{")]
        assert p.returncode == 0 and lines, (p.returncode, out[-2000:], err[-4000:])
        results.append(json.loads(lines[-1]))
    assert all(r["ok"] for r in results), results


def test_put_wait_times_out_without_peer(ocean):
    """Rank 0 of two issues its frame alone: its row pass waits for rank 1's blocks, which never come.
    The wait gives up after the timeout (every wave exits), the stream drains, and
    ocean_peers_synchronize reports OCEAN_ERR_TIMEOUT."""
    import time

    from oceansimulation_amd import capi
    from oceansimulation_amd.capi import OceanError
    from oceansimulation_amd.slab import PeerExchange, SlabGenerator

    n = 8192
    fft = ocean.FFTCalculator(n)
    slabs = [SlabGenerator(fft, r, 2) for r in range(2)]
    peers = [PeerExchange(g) for g in slabs]
    PeerExchange.connect_local(peers)
    peers[0].set_timeout(300)
    t0 = time.perf_counter()
    slabs[0].put_columns(peers[0], 0.5, True)
    slabs[0].put_rows(peers[0])
    with pytest.raises(OceanError) as exc:
        peers[0].synchronize()
    assert exc.value.code == capi.OCEAN_ERR_TIMEOUT
    assert "ready" in str(exc.value)
    assert time.perf_counter() - t0 < 30.0
    for p in peers:
        p.close()
    for g in slabs:
        g.close()
    fft.close()


def test_comm_wrap_checks_size_and_rank(ocean):
    """ocean_comm_wrap takes the caller's ncclComm_t only when nranks / rank are the communicator's own
    (ncclCommCount / ncclCommUserRank): a one-rank RCCL communicator made here (through the RCCL that
    liboceanfft.so links, resolved via the library's own handle) is refused as rank 1 of 2 and taken as
    rank 0 of 1."""
    import ctypes

    from oceansimulation_amd import capi

    L = capi.lib()

    class UniqueId(ctypes.Structure):
        _fields_ = [("internal", ctypes.c_char * capi.OCEAN_COMM_ID_BYTES)]

    get_id, init_rank, destroy = L.ncclGetUniqueId, L.ncclCommInitRank, L.ncclCommDestroy
    get_id.argtypes, get_id.restype = [ctypes.POINTER(UniqueId)], ctypes.c_int
    init_rank.argtypes = [ctypes.POINTER(ctypes.c_void_p), ctypes.c_int, UniqueId, ctypes.c_int]
    init_rank.restype = ctypes.c_int
    destroy.argtypes, destroy.restype = [ctypes.c_void_p], ctypes.c_int
    uid = UniqueId()
    assert get_id(ctypes.byref(uid)) == 0
    nc = ctypes.c_void_p()
    assert init_rank(ctypes.byref(nc), 1, uid, 0) == 0
    wrapped = ctypes.c_void_p()
    assert L.ocean_comm_wrap(ctypes.byref(wrapped), nc, 2, 1) == capi.OCEAN_ERR_INVALID
    assert "rank 0 of 1" in L.ocean_last_error().decode()
    assert not wrapped.value
    assert L.ocean_comm_wrap(ctypes.byref(wrapped), nc, 1, 0) == capi.OCEAN_OK
    assert wrapped.value
    assert L.ocean_comm_destroy(wrapped) == capi.OCEAN_OK  # a wrapped communicator stays the caller's
    assert destroy(nc) == 0
