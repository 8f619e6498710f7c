"""Latency/bandwidth floor at the bench's sizes: an empty launch and a one-round-trip
tile copy that moves exactly the encode / reconstruct bytes per tile of 8 trajectories.
    python tools/floor/floor.py
"""
import ctypes as C
import json
import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, REPO)


def main():
    import torch
    from bench import kernel_time_us
    so = os.path.join(HERE, "libfloor.so")
    subprocess.run(["hipcc", "-O3", "--offload-arch=gfx950", "-shared", "-fPIC", "-o", so,
                    os.path.join(HERE, "floor.hip")], check=True)
    lib = C.CDLL(so)
    lib.floor_empty.argtypes = [C.c_int, C.c_void_p]
    lib.floor_tile_copy.argtypes = [C.c_void_p, C.c_int64, C.c_void_p, C.c_int64, C.c_int64, C.c_int, C.c_void_p]
    dev = torch.device("cuda", 0)
    s = torch.cuda.current_stream(dev)
    out = {"empty_1": kernel_time_us(lambda: lib.floor_empty(1, s.cuda_stream), s, 50),
           "empty_512": kernel_time_us(lambda: lib.floor_empty(512, s.cuda_stream), s, 50)}
    # encode tile: 8 x 50 x 14 f32 in (22400 B), 8 x 140 (f32 + i64) out (13440 B)
    # reconstruct tile: 8 x 140 i64 in (8960 B), 8 x 50 x 14 f32 out (22400 B)
    for B in (4096, 65536, 1048576):
        nt = B // 8
        for name, ib, ob in (("enc", 22400, 13440), ("rec", 8960, 22400)):
            x = torch.empty(nt * ib // 4, dtype=torch.float32, device=dev).fill_(1)
            y = torch.empty(nt * ob // 4, dtype=torch.float32, device=dev)
            for grid in sorted({min(nt, g) for g in (nt, 1024, 2048)}):
                us = kernel_time_us(lambda: lib.floor_tile_copy(x.data_ptr(), ib // 16, y.data_ptr(), ob // 16, nt,
                                                                grid, s.cuda_stream), s, 30)
                out[f"{name}_B{B}_grid{grid}"] = {"us": round(us, 2),
                                                  "GBs": round(nt * (ib + ob) / us / 1e3, 1)}
            del x, y
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
