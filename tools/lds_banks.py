#!/usr/bin/env python3
"""LDS bank-conflict model of fft_run's exchanges (device/fft.h) for the row pass (k_rows_half):
every ds_write_b64 / ds_read_b64 a wave issues, banked per MI355X_MICROARCH.md §LDS (read_b64: 2
groups of 32 lanes, bank = dword mod 64; write_b64 / write2_b64: 4 groups of 16 lanes, bank = dword
mod 32). Extra cycles = sum over groups of (max distinct addresses on one bank - 1). Compares the row
layout (CI = 0: regions RPW apart by PADDED + 4) with interleaved regions (CI = RPW) and the lane
order of the post-exchange mapping. Usage: python tools/lds_banks.py"""
import collections


def shape(logn):
    n = 1 << logn
    t = n >> 4
    lr0 = (logn & 3) or 4
    return n, t, 1 << lr0, 1 + (logn - lr0) // 4, n + n // 16


def pad16(a):
    return a + (a >> 4)


def read_pidx(logn, i, m):
    n, t, r0, ns, padded = shape(logn)
    return pad16(i) + m * (t + t // 16) if (t & 15) == 0 else pad16(i + m * t)


def slot(ci, padded, reg, pa):
    return pa * ci + reg if ci > 0 else reg * (padded + 4) + pa


def exchanges(logn, lanes_load, lanes_post):
    """Yield (kind, per-lane slot list) for every write/read instruction of one fft_run.
    lanes_load[l] = (i, reg) before the first exchange, lanes_post[l] = (i2, reg2) after."""
    n, t, r0, ns, padded = shape(logn)
    # stage 0 writes
    if r0 == 16:
        yield "w", [[17 * i + tt for (i, reg) in lanes_load] for tt in range(16)], [reg for (i, reg) in lanes_load]
    else:
        u_ = 16 // r0
        def wp(i, q):
            u, tt = q % u_, q // u_
            return pad16((i + u * t) * r0 + tt)
        yield "w", [[wp(i, q) for (i, reg) in lanes_load] for q in range(16)], [reg for (i, reg) in lanes_load]
    yield "r", [[read_pidx(logn, i2, m) for (i2, r2) in lanes_post] for m in range(16)], [r2 for (i2, r2) in lanes_post]
    p = r0
    for s in range(1, ns):
        if s + 1 < ns:
            def wp2(i2, tt, p=p):
                k = i2 & (p - 1)
                j = (i2 // p) * 16 * p + k
                return pad16(j) + tt * (p + p // 16) if p >= 16 else pad16(j + tt * p)
            yield "w", [[wp2(i2, tt) for (i2, r2) in lanes_post] for tt in range(16)], [r2 for (i2, r2) in lanes_post]
            yield "r", [[read_pidx(logn, i2, m) for (i2, r2) in lanes_post] for m in range(16)], [r2 for (i2, r2) in lanes_post]
        p *= 16


def conflicts(kind, slots_by_lane):
    """Extra LDS cycles of one wave instruction (8-byte elements)."""
    groups = [range(0, 32), range(32, 64)] if kind == "r" else [range(g * 16, g * 16 + 16) for g in range(4)]
    nbank = 64 if kind == "r" else 32
    extra = 0
    for g in groups:
        banks = collections.defaultdict(set)
        for l in g:
            for d in (2 * slots_by_lane[l], 2 * slots_by_lane[l] + 1):
                banks[d % nbank].add(d)
        extra += max(len(v) for v in banks.values()) - 1
    return extra


def run(logn, rpw, ci, post_order):
    n, t, r0, ns, padded = shape(logn)
    wg = t * rpw
    b_ = 4  # ColFirstCfg B for the half path (N = 1024 .. 4096)
    total, count = 0, 0
    for w0 in range(0, wg, 64):
        lanes_load, lanes_post = [], []
        for tid in range(w0, w0 + 64):
            b, r, ihi = tid % b_, (tid // b_) % rpw, tid // (b_ * rpw)
            lanes_load.append((ihi * b_ + b, r))
            if post_order == "row":  # i2 fastest (one row per wave)
                lanes_post.append((tid % t, tid // t))
            else:  # r2 fastest (the RPW rows interleaved)
                lanes_post.append(((tid // rpw) % t, tid % rpw))
        for kind, per_instr, regs in exchanges(logn, lanes_load, lanes_post):
            for pas in per_instr:
                sl = [slot(ci, padded, reg, pa) for pa, reg in zip(pas, regs)]
                total += conflicts(kind, sl)
                count += 1
    return total, count


if __name__ == "__main__":
    for logn in (10, 11, 12):
        for ci, order, name in ((0, "row", "row layout, i2 fastest (round 1)"), (2, "interleaved", "interleaved regions, r2 fastest")):
            extra, cnt = run(logn, 2, ci, order)
            print(f"N={1 << logn:5d} RPW=2 {name:36s}: {extra:5d} extra LDS cycles over {cnt} wave instructions")
