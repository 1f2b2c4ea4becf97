#!/usr/bin/env python3
"""Run the PMC calibration kernels (tools/pmc_calib.hip) over a 1 GiB buffer.

Under `rocprofv3 --pmc FETCH_SIZE` (and separately WRITE_SIZE) each dispatch moves a
known 1 GiB, giving the counter -> bytes factor for 4-B and 16-B per-lane accesses.
"""
import ctypes
import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
SRC = os.path.join(HERE, "pmc_calib.hip")
LIB = os.path.join(HERE, "_lib", "libpmccalib.so")
BYTES = 1 << 30


def build():
    os.makedirs(os.path.dirname(LIB), exist_ok=True)
    if not os.path.exists(LIB) or os.path.getmtime(LIB) < os.path.getmtime(SRC):
        subprocess.check_call(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-fPIC", "-shared",
                               "-o", LIB, SRC])


def main():
    build()
    if len(sys.argv) > 1 and sys.argv[1] == "build":
        return
    import torch
    lib = ctypes.CDLL(LIB)
    lib.pmc_calib_run.argtypes = [ctypes.c_void_p, ctypes.c_int64, ctypes.c_void_p]
    buf = torch.ones(BYTES // 4, dtype=torch.int32, device="cuda:0")
    sink = torch.zeros(16, dtype=torch.int32, device="cuda:0")
    torch.cuda.synchronize()
    for _ in range(3):
        assert lib.pmc_calib_run(buf.data_ptr(), BYTES, sink.data_ptr()) == 0
    print("pmc calib done: 3 x {read_dword, read_dwordx4, write_dword, write_dwordx4} over %d bytes" % BYTES)


if __name__ == "__main__":
    main()
