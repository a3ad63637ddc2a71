"""Slab decomposition of one N x N cascade over several GPUs.

Rank r of P runs the column pass on columns [r*w, r*w + w) and the row pass on rows
[r*w, r*w + w), w = N/P. Between them a single equal-split all-to-all moves block q of every
rank's column-pass output to rank q (include/oceanfft.h, "slab decomposition"). The reference
runs one cascade on one device; this is the multi-GPU extension of its CalculateOcean.

Frames are independent until their exchange (the column pass depends only on h0 and t), so
`SlabPipeline` overlaps frame f's all-to-all with frame f+1's column pass and frame f-1's row
pass (two buffer slots, the exchange on its own stream); steady state is max(exchange, passes)
instead of their sum. Maps then lag the last issued frame by one until `flush()`.

Four exchanges are provided:
  * `PeerExchange` + `SlabGenerator.frame_put` / `frame_put_pipelined`: the one-sided exchange of
    the C ABI (ocean_peers, four-step slabs): the column pass stores each destination block straight
    into the owning rank's receive slot through an IPC mapping of its memory, and one flag word per
    rank and frame replaces the collective — no send buffer, no copy kernel;
  * `RcclComm` + `SlabGenerator.frame` / `frame_pipelined`: the library's own all-to-all, grouped
    ncclSend / ncclRecv over RCCL inside the C ABI (ocean_generator_slab_frame[_pipelined]), one
    process per GPU — used by bench.py;
  * `TorchExchange`: torch.distributed.all_to_all_single over the "nccl" backend (RCCL on ROCm), the
    comparator leg and the one-GPU gloo rehearsal;
  * `emulate_frame`: P slab generators in one process/GPU, blocks moved by device copies — used by
    the parity tests to check the decomposition against the whole-grid generator.
"""
from __future__ import annotations

import ctypes

import numpy as np

from . import hip
from .capi import OceanError, OceanSettings, check, lib
from .waves import FFTCalculator


class SlabGenerator:
    """One rank's part of a single N x N grid (ocean_generator_create_slab)."""

    def __init__(self, fft: FFTCalculator, rank: int, ranks: int):
        h = ctypes.c_void_p()
        check(lib().ocean_generator_create_slab(ctypes.byref(h), fft.handle, rank, ranks),
              "ocean_generator_create_slab")
        self._h = h
        self.fft = fft
        self.n = fft.GetTextureResolution()
        self.rank, self.ranks = rank, ranks
        self.rows = self.n // ranks
        self.row0 = rank * self.rows

    @property
    def exchange_bytes(self) -> int:
        """Bytes of this rank's send (and receive) buffer: ranks equal blocks."""
        return int(lib().ocean_generator_exchange_bytes(self._h))

    def set_half_spectrum(self, enable: bool) -> None:
        """Strip-dealt half-spectrum path (default for N >= 1024) or the full-spectrum path; the
        exchange size changes with it and h0 is re-seeded at the next frame."""
        check(lib().ocean_generator_set_half_spectrum(self._h, 1 if enable else 0), "ocean_generator_set_half_spectrum")

    def set_four_step(self, enable: bool) -> None:
        """N = 8192 / 16384: the four-step column pass writing destination-block order (default; the
        row pass reads the received blocks directly) or the strip-dealt column pass + transposes.
        Changes exchange_bytes."""
        check(lib().ocean_generator_set_four_step(self._h, 1 if enable else 0), "ocean_generator_set_four_step")

    def frame_bytes(self):
        """Algorithmic HBM bytes per point of the column pass and the row pass (transposes included)."""
        b = (ctypes.c_double * 2)()
        check(lib().ocean_generator_frame_bytes(self._h, b), "ocean_generator_frame_bytes")
        return b[0], b[1]

    @property
    def handle(self):
        return self._h

    def GetOceanSettings(self) -> OceanSettings:
        p = lib().ocean_generator_settings(self._h, 0)
        if not p:
            raise OceanError(1, "ocean_generator_settings")
        return p.contents

    def columns(self, timestep: float, update_ocean: bool = False, send_ptr: int | None = None) -> None:
        check(lib().ocean_generator_slab_columns(self._h, ctypes.c_float(timestep), 1 if update_ocean else 0,
                                                 ctypes.c_void_p(send_ptr or 0)), "ocean_generator_slab_columns")

    def rows_pass(self, recv_ptr: int | None = None) -> None:
        check(lib().ocean_generator_slab_rows(self._h, ctypes.c_void_p(recv_ptr or 0)), "ocean_generator_slab_rows")

    def frame(self, comm: "RcclComm", timestep: float, update_ocean: bool = False) -> None:
        """Columns, the RCCL all-to-all and rows, all inside the library (ocean_generator_slab_frame)."""
        check(lib().ocean_generator_slab_frame(self._h, comm.handle, ctypes.c_float(timestep), 1 if update_ocean else 0),
              "ocean_generator_slab_frame")

    def frame_pipelined(self, comm: "RcclComm", timestep: float, update_ocean: bool = False) -> None:
        """Frame f's all-to-all on the library's comm stream beside frame f + 1's column pass and frame
        f - 1's row pass; the maps lag by one frame until flush()."""
        check(lib().ocean_generator_slab_frame_pipelined(self._h, comm.handle, ctypes.c_float(timestep),
                                                         1 if update_ocean else 0), "ocean_generator_slab_frame_pipelined")

    def flush(self) -> None:
        check(lib().ocean_generator_slab_flush(self._h), "ocean_generator_slab_flush")

    def frame_put(self, peers: "PeerExchange", timestep: float, update_ocean: bool = False) -> None:
        """One frame over the one-sided exchange (ocean_generator_slab_frame_put)."""
        check(lib().ocean_generator_slab_frame_put(self._h, peers.handle, ctypes.c_float(timestep),
                                                   1 if update_ocean else 0), "ocean_generator_slab_frame_put")

    def frame_put_pipelined(self, peers: "PeerExchange", timestep: float, update_ocean: bool = False) -> None:
        """Frame f's column pass and put on the peers' stream beside frame f - 1's row pass; the maps lag
        by one frame until peers.flush()."""
        check(lib().ocean_generator_slab_frame_put_pipelined(self._h, peers.handle, ctypes.c_float(timestep),
                                                             1 if update_ocean else 0),
              "ocean_generator_slab_frame_put_pipelined")

    def put_columns(self, peers: "PeerExchange", timestep: float, update_ocean: bool = False) -> None:
        check(lib().ocean_generator_slab_put_columns(self._h, peers.handle, ctypes.c_float(timestep),
                                                     1 if update_ocean else 0), "ocean_generator_slab_put_columns")

    def put_rows(self, peers: "PeerExchange") -> None:
        check(lib().ocean_generator_slab_put_rows(self._h, peers.handle), "ocean_generator_slab_put_rows")

    def height_map_host(self) -> np.ndarray:
        self.fft.synchronize()
        return hip.to_host(int(lib().ocean_generator_height_map(self._h, 0)), (self.rows, self.n, 4))

    def displacement_map_host(self) -> np.ndarray:
        self.fft.synchronize()
        return hip.to_host(int(lib().ocean_generator_displacement_map(self._h, 0)), (self.rows, self.n, 4))

    def jacobian_map_host(self) -> np.ndarray:
        self.fft.synchronize()
        return hip.to_host(int(lib().ocean_generator_jacobian_map(self._h, 0)), (self.rows, self.n))

    def set_profiling(self, enable: bool) -> None:
        check(lib().ocean_generator_set_profiling(self._h, 1 if enable else 0), "ocean_generator_set_profiling")

    def kernel_times(self):
        ms = (ctypes.c_double * 3)()
        cnt = (ctypes.c_int64 * 3)()
        check(lib().ocean_generator_kernel_times(self._h, ms, cnt), "ocean_generator_kernel_times")
        return list(ms), list(cnt)

    def kernel_times4(self):
        """kernel_times with index 3 = the put of one-sided frames (inside index 1)."""
        ms = (ctypes.c_double * 4)()
        cnt = (ctypes.c_int64 * 4)()
        check(lib().ocean_generator_kernel_times4(self._h, ms, cnt), "ocean_generator_kernel_times4")
        return list(ms), list(cnt)

    def close(self) -> None:
        if self._h:
            lib().ocean_generator_destroy(self._h)
            self._h = ctypes.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class RcclComm:
    """The C ABI's RCCL communicator over the P ranks of one grid (ocean_comm_create). Rank 0's unique
    id reaches the other ranks through `share_id(bytes) -> bytes` (e.g. a torch.distributed broadcast)."""

    def __init__(self, rank: int, ranks: int, share_id):
        from .capi import OCEAN_COMM_ID_BYTES

        uid = (ctypes.c_ubyte * OCEAN_COMM_ID_BYTES)()
        if rank == 0:
            check(lib().ocean_comm_unique_id(uid), "ocean_comm_unique_id")
        got = share_id(bytes(uid))
        uid = (ctypes.c_ubyte * OCEAN_COMM_ID_BYTES).from_buffer_copy(got)
        h = ctypes.c_void_p()
        check(lib().ocean_comm_create(ctypes.byref(h), uid, ranks, rank), "ocean_comm_create")
        self._h = h

    @property
    def handle(self):
        return self._h

    def all_to_all(self, send_ptr: int, recv_ptr: int, nbytes: int, stream: int | None = None) -> None:
        """Equal-split all-to-all of device buffers (ocean_comm_all_to_all), enqueued on `stream`."""
        check(lib().ocean_comm_all_to_all(self._h, ctypes.c_void_p(send_ptr), ctypes.c_void_p(recv_ptr), nbytes,
                                          ctypes.c_void_p(stream or 0)), "ocean_comm_all_to_all")

    def close(self) -> None:
        if self._h:
            lib().ocean_comm_destroy(self._h)
            self._h = ctypes.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class PeerExchange:
    """The one-sided slab exchange of one rank (ocean_peers): two receive slots and the flag words in
    this process's device memory. connect(gather) hands this rank's handle to `gather(bytes) -> list of
    bytes in rank order` (e.g. a torch.distributed all_gather_object) and maps the others'; or
    connect_local(...) for P ranks of one process (the one-GPU emulation). Before close(), every rank
    must have synchronized and passed a host barrier: a peer may still signal into this rank's flags."""

    def __init__(self, gen: SlabGenerator):
        h = ctypes.c_void_p()
        check(lib().ocean_peers_create(ctypes.byref(h), gen.handle), "ocean_peers_create")
        self._h = h
        self.gen = gen

    @property
    def handle(self):
        return self._h

    def exported(self) -> bytes:
        from .capi import OCEAN_PEER_HANDLE_BYTES

        buf = (ctypes.c_ubyte * OCEAN_PEER_HANDLE_BYTES)()
        check(lib().ocean_peers_handle(self._h, buf), "ocean_peers_handle")
        return bytes(buf)

    def connect(self, gather) -> None:
        handles = b"".join(gather(self.exported()))
        buf = (ctypes.c_ubyte * len(handles)).from_buffer_copy(handles)
        check(lib().ocean_peers_connect(self._h, buf), "ocean_peers_connect")

    @staticmethod
    def connect_local(peers) -> None:
        arr = (ctypes.c_void_p * len(peers))(*[p.handle.value for p in peers])
        check(lib().ocean_peers_connect_local(arr, len(peers)), "ocean_peers_connect_local")

    def set_timeout(self, ms: int) -> None:
        check(lib().ocean_peers_set_timeout(self._h, int(ms)), "ocean_peers_set_timeout")

    def set_put_cus(self, cus: int) -> None:
        check(lib().ocean_peers_set_put_cus(self._h, int(cus)), "ocean_peers_set_put_cus")

    def set_streams(self, column_stream: int | None, put_stream: int | None, row_stream: int | None) -> None:
        """Streams of pipelined frames' step 1, put and row pass (None: the peers' own)."""
        check(lib().ocean_peers_set_streams(self._h, ctypes.c_void_p(column_stream or 0), ctypes.c_void_p(put_stream or 0),
                                            ctypes.c_void_p(row_stream or 0)), "ocean_peers_set_streams")

    def set_row_cus(self, cus: int) -> None:
        """The CUs the caller's (CU-masked) row stream may use: sizes the resident row-pass grid (0: all)."""
        check(lib().ocean_peers_set_row_cus(self._h, int(cus)), "ocean_peers_set_row_cus")

    def set_put_cu_mask(self, cus_per_xcd: int) -> None:
        """CU-mask the peers' own streams: the put on `cus_per_xcd` CUs of every XCD, step 1 and rows on
        the others (0: unmasked)."""
        check(lib().ocean_peers_set_put_cu_mask(self._h, int(cus_per_xcd)), "ocean_peers_set_put_cu_mask")

    def flush(self) -> None:
        check(lib().ocean_peers_flush(self._h), "ocean_peers_flush")

    def debug_slot(self, slot: int):
        """(device pointer, bytes) of receive slot `slot` (frame f lands in slot f % 2); debug only."""
        ptr, nbytes = ctypes.c_void_p(), ctypes.c_size_t()
        check(lib().ocean_peers_debug_slot(self._h, int(slot), ctypes.byref(ptr), ctypes.byref(nbytes)),
              "ocean_peers_debug_slot")
        return int(ptr.value), int(nbytes.value)

    def synchronize(self) -> None:
        """Wait for this rank's streams; raises OceanError (OCEAN_ERR_TIMEOUT) when a wait gave up."""
        check(lib().ocean_peers_synchronize(self._h), "ocean_peers_synchronize")

    def close(self) -> None:
        if self._h:
            lib().ocean_peers_destroy(self._h)
            self._h = ctypes.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def torch_gather_bytes(blob: bytes):
    """All-gather one bytes object per rank over the default torch.distributed group (rank order)."""
    import torch.distributed as dist

    if not (dist.is_available() and dist.is_initialized()) or dist.get_world_size() == 1:
        return [blob]
    out = [None] * dist.get_world_size()
    dist.all_gather_object(out, blob)
    return out


def emulate_put_frame(slabs, peers, timestep: float, update_ocean: bool = False) -> None:
    """One frame of a P-rank slab grid inside one process over the one-sided exchange (peers joined
    by PeerExchange.connect_local): every rank's column pass stores into the others' slots, then every
    rank's row pass reads its own."""
    for g, p in zip(slabs, peers):
        g.put_columns(p, timestep, update_ocean)
    for g, p in zip(slabs, peers):
        g.put_rows(p)


def torch_share_id(uid: bytes) -> bytes:
    """Broadcast rank 0's communicator id over the default torch.distributed group (any backend)."""
    import torch.distributed as dist

    if not (dist.is_available() and dist.is_initialized()) or dist.get_world_size() == 1:
        return uid
    box = [uid]
    dist.broadcast_object_list(box, src=0)
    return box[0]


def slab_layout(n: int, rank: int, ranks: int, half=True):
    """ocean_slab_layout: half = True / 1: the strip-dealt path (first strip, strips, strip slots per
    block, rows, block bytes, exchange bytes); 2: the four-step path (first kept column, kept columns,
    holds the Nyquist column, rows, block bytes, exchange bytes); False / 0: the full spectrum. Host
    only, no device needed."""
    out = (ctypes.c_int64 * 6)()
    check(lib().ocean_slab_layout(n, rank, ranks, int(half), out), "ocean_slab_layout")
    return tuple(int(v) for v in out)


def block_moves(ranks: int, nbytes: int):
    """(src_rank, src_offset, dst_rank, dst_offset, size) of the equal-split all-to-all."""
    blk = nbytes // ranks
    return [(s, q * blk, q, s * blk, blk) for s in range(ranks) for q in range(ranks)]


def emulate_frame(slabs, sends, recvs, timestep: float, update_ocean: bool = False) -> None:
    """One frame of a P-rank slab grid inside one process: columns, device-copy exchange, rows."""
    for g, snd in zip(slabs, sends):
        g.columns(timestep, update_ocean, snd.ptr)
    hip.synchronize()
    for s, so, q, qo, size in block_moves(len(slabs), slabs[0].exchange_bytes):
        hip.copy_d2d(recvs[q].ptr + qo, sends[s].ptr + so, size)
    for g, rcv in zip(slabs, recvs):
        g.rows_pass(rcv.ptr)


def _staged() -> bool:
    """gloo (CPU collectives) is used only to rehearse several ranks on one GPU (bench.py
    --shared-gpu): device buffers then go through host memory."""
    import torch.distributed as dist

    return dist.get_backend() == "gloo"


def _all_to_all(recv, send, stream=None) -> None:
    import torch
    import torch.distributed as dist

    if not _staged():
        dist.all_to_all_single(recv, send)
        return
    host_send = send.to("cpu", non_blocking=False)
    host_recv = torch.empty_like(host_send)
    dist.all_to_all_single(host_recv, host_send)
    recv.copy_(host_recv, non_blocking=False)


class TorchExchange:
    """Equal-split all-to-all over torch.distributed (backend "nccl" = RCCL on ROCm)."""

    def __init__(self, nbytes: int, device):
        import torch

        self.send = torch.empty(nbytes, dtype=torch.uint8, device=device)
        self.recv = torch.empty(nbytes, dtype=torch.uint8, device=device)

    def __call__(self) -> None:
        _all_to_all(self.recv, self.send)


class SlabPipeline:
    """Software pipeline of slab frames over two send/recv buffer slots.

    step(dt), frame f, slot s = f % 2:
      compute stream:  columns(f) -> send[s]; record cols_done[s]
      comm stream:     wait cols_done[s], rows_done[s] (row pass f-2 has finished reading recv[s]);
                       exchange(s): send[s] -> recv[s]; record xchg_done[s]
      compute stream:  wait xchg_done[1-s]; rows(f-1) from recv[1-s]; record rows_done[1-s]
    The compute stream is the generators' stream (their ocean_fft's); columns(f+2) reuses send[s]
    only after rows(f) was issued behind xchg_done[s], so in-order execution protects it.
    `exchange(slot, comm_stream)` must enqueue the data movement of slot `slot` on `comm_stream`
    (TorchExchangeSlots for RCCL across processes, LocalExchangeSlots for ranks in one process).
    """

    def __init__(self, gens, send_ptrs, recv_ptrs, exchange, compute_stream=None):
        import torch

        self.gens = list(gens)
        self.send, self.recv = send_ptrs, recv_ptrs  # [slot][gen] device pointers
        self.exchange = exchange
        self.compute = compute_stream if compute_stream is not None else torch.cuda.default_stream()
        self.comm = torch.cuda.Stream(device=self.compute.device)
        self.cols_done = [torch.cuda.Event() for _ in range(2)]
        self.xchg_done = [torch.cuda.Event() for _ in range(2)]
        self.rows_done = [torch.cuda.Event() for _ in range(2)]
        self.rows_recorded = [False, False]
        self.pending = None  # slot whose row pass is still to be issued
        self.frame = 0

    def step(self, timestep: float, update_ocean: bool = False) -> None:
        s = self.frame % 2
        for k, g in enumerate(self.gens):
            g.columns(timestep, update_ocean, self.send[s][k])
        self.cols_done[s].record(self.compute)
        self.comm.wait_event(self.cols_done[s])
        if self.rows_recorded[s]:
            self.comm.wait_event(self.rows_done[s])
        self.exchange(s, self.comm)
        self.xchg_done[s].record(self.comm)
        if self.pending is not None:
            self._rows(self.pending)
        self.pending = s
        self.frame += 1

    def _rows(self, s: int) -> None:
        self.compute.wait_event(self.xchg_done[s])
        for k, g in enumerate(self.gens):
            g.rows_pass(self.recv[s][k])
        self.rows_done[s].record(self.compute)
        self.rows_recorded[s] = True

    def flush(self) -> None:
        """Issue the last frame's row pass: afterwards the maps hold the last stepped frame."""
        if self.pending is not None:
            self._rows(self.pending)
            self.pending = None


class LocalExchangeSlots:
    """Exchange for P slab generators in one process (tests): two slots of per-rank send/recv
    buffers, the equal-split block moves as device copies on the comm stream. The multi-process
    path is TorchExchangeSlots."""

    def __init__(self, ranks: int, nbytes: int, device):
        import torch

        self.send = [[torch.empty(nbytes, dtype=torch.uint8, device=device) for _ in range(ranks)] for _ in range(2)]
        self.recv = [[torch.empty(nbytes, dtype=torch.uint8, device=device) for _ in range(ranks)] for _ in range(2)]
        self.moves = block_moves(ranks, nbytes)

    def ptrs(self):
        return ([[t.data_ptr() for t in slot] for slot in self.send],
                [[t.data_ptr() for t in slot] for slot in self.recv])

    def __call__(self, slot: int, stream) -> None:
        import torch

        with torch.cuda.stream(stream):
            for src, so, dst, do, size in self.moves:
                self.recv[slot][dst][do:do + size].copy_(self.send[slot][src][so:so + size], non_blocking=True)


class TorchExchangeSlots:
    """Two slots of equal-split all-to-all over torch.distributed ("nccl" = RCCL on ROCm). The
    collective is issued asynchronously from the comm stream, which then waits for it."""

    def __init__(self, nbytes: int, device):
        import torch

        self.send = [torch.empty(nbytes, dtype=torch.uint8, device=device) for _ in range(2)]
        self.recv = [torch.empty(nbytes, dtype=torch.uint8, device=device) for _ in range(2)]

    def ptrs(self):
        return [[t.data_ptr()] for t in self.send], [[t.data_ptr()] for t in self.recv]

    def __call__(self, slot: int, stream) -> None:
        import torch
        import torch.distributed as dist

        with torch.cuda.stream(stream):
            if _staged():  # rehearsal on one GPU: host-staged and synchronous
                _all_to_all(self.recv[slot], self.send[slot])
                return
            work = dist.all_to_all_single(self.recv[slot], self.send[slot], async_op=True)
            work.wait()  # comm stream waits for the collective; the host does not block
