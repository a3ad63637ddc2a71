"""Slab decomposition of one N x N cascade over several GPUs.

Rank r of P runs the column pass on columns [r*w, r*w + w) and the row pass on rows
[r*w, r*w + w), w = N/P. Between them a single equal-split all-to-all moves block q of every
rank's column-pass output to rank q (include/oceanfft.h, "slab decomposition"). The reference
runs one cascade on one device; this is the multi-GPU extension of its CalculateOcean.

Two exchanges are provided:
  * `TorchExchange`: torch.distributed.all_to_all_single over the "nccl" backend (RCCL on ROCm),
    one process per GPU — used by bench.py;
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
        self.exchange_bytes = int(lib().ocean_generator_exchange_bytes(self._h))

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

    def close(self) -> None:
        if self._h:
            lib().ocean_generator_destroy(self._h)
            self._h = ctypes.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


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


class TorchExchange:
    """Equal-split all-to-all over torch.distributed (backend "nccl" = RCCL on ROCm)."""

    def __init__(self, nbytes: int, device):
        import torch

        self.send = torch.empty(nbytes, dtype=torch.uint8, device=device)
        self.recv = torch.empty(nbytes, dtype=torch.uint8, device=device)

    def __call__(self) -> None:
        import torch.distributed as dist

        dist.all_to_all_single(self.recv, self.send)
