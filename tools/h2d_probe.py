"""Host-to-device rates of a memory-mapped capture file (GPU box): can the reader's read-only file map be page-locked
(hipHostRegister) and DMA'd from directly, and how do pageable hipMemcpy, a registered map and a copy into page-locked
staging compare?  Decides whether the file path may skip its staging copy (the file path).

  python tools/h2d_probe.py [MiB]
"""
from __future__ import annotations

import ctypes
import mmap
import os
import sys
import time

import numpy as np
import torch


def main() -> None:
    mib = int(sys.argv[1]) if len(sys.argv) > 1 else 1024
    size = mib << 20
    torch.zeros(1, device="cuda:0")
    hip = ctypes.CDLL("libamdhip64.so")
    hip.hipHostRegister.argtypes = [ctypes.c_void_p, ctypes.c_size_t, ctypes.c_uint]
    hip.hipHostUnregister.argtypes = [ctypes.c_void_p]
    hip.hipMemcpy.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int]
    path = f"/dev/shm/pcppx_h2d_{os.getpid()}.bin"
    dev = torch.empty(size, dtype=torch.uint8, device="cuda:0")
    try:
        with open(path, "wb") as f:
            f.write(np.random.default_rng(1).integers(0, 256, size, dtype=np.uint8).tobytes())
        fd = os.open(path, os.O_RDONLY)
        m = mmap.mmap(fd, size, flags=mmap.MAP_PRIVATE, prot=mmap.PROT_READ)
        os.close(fd)
        arr = np.frombuffer(m, dtype=np.uint8)
        addr = arr.ctypes.data
        _ = int(arr[:: 4096].sum())  # fault the map in (as the reader's record walk does)

        def h2d(src) -> float:
            torch.cuda.synchronize()
            t = time.perf_counter()
            rc = hip.hipMemcpy(ctypes.c_void_p(dev.data_ptr()), ctypes.c_void_p(src), size, 1)
            torch.cuda.synchronize()
            assert rc == 0, rc
            return size / (time.perf_counter() - t) / 1e9

        print(f"pageable map -> HBM: {max(h2d(addr) for _ in range(3)):.1f} GB/s", flush=True)
        t = time.perf_counter()
        rc = hip.hipHostRegister(ctypes.c_void_p(addr), size, 0)
        reg_s = time.perf_counter() - t
        print(f"hipHostRegister(read-only private file map, {mib} MiB): rc={rc} in {reg_s * 1e3:.1f} ms "
              f"({size / reg_s / 1e9:.1f} GB/s)", flush=True)
        if rc == 0:
            print(f"registered map -> HBM: {max(h2d(addr) for _ in range(3)):.1f} GB/s", flush=True)
            ok = torch.equal(dev[:: 65536].cpu(), torch.from_numpy(arr[:: 65536].copy()))
            print(f"bytes equal: {ok}", flush=True)
            t = time.perf_counter()
            hip.hipHostUnregister(ctypes.c_void_p(addr))
            print(f"hipHostUnregister: {(time.perf_counter() - t) * 1e3:.1f} ms", flush=True)
        pinned = torch.empty(size, dtype=torch.uint8, pin_memory=True)
        t = time.perf_counter()
        pinned.numpy()[:] = arr
        cp = time.perf_counter() - t
        print(f"copy map -> page-locked staging (1 thread): {size / cp / 1e9:.1f} GB/s; staging -> HBM: "
              f"{max(h2d(pinned.data_ptr()) for _ in range(3)):.1f} GB/s", flush=True)
        del arr
        m.close()
    finally:
        os.unlink(path)


if __name__ == "__main__":
    main()
