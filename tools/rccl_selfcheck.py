"""RCCL self-exchange check (world size 1): ocean_comm_all_to_all of random buffers of growing size
through the C ABI's communicator must copy them exactly. Found RCCL 2.26 corrupting single sends /
receives above 1 GiB (profiles/r03_rccl_selfcheck.log, before the exchange was cut into 512-MiB
pieces). Usage on a GPU box: python tools/rccl_selfcheck.py"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from oceansimulation_amd.slab import RcclComm  # noqa: E402

comm = RcclComm(0, 1, lambda u: u)
for mb in (1, 64, 512, 1024, 1400, 2100, 3000):
    n = mb << 20
    a = torch.randint(0, 255, (n,), dtype=torch.uint8, device="cuda")
    b = torch.zeros_like(a)
    comm.all_to_all(a.data_ptr(), b.data_ptr(), n, 0)
    torch.cuda.synchronize()
    eq = bool(torch.equal(a, b))
    print(f"{mb} MiB: equal={eq}", flush=True)
    del a, b
    torch.cuda.empty_cache()
comm.close()
