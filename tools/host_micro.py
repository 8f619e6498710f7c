"""Cost of each host-side piece of an encode call (ctypes, allocation, stream query ...)."""
import json
import os
import sys
import time

import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
from beast_tokenizer_amd import _lib  # noqa: E402


def t(fn, n=20000):
    for _ in range(200):
        fn()
    t0 = time.perf_counter()
    for _ in range(n):
        fn()
    return round((time.perf_counter() - t0) / n * 1e6, 3)


dev = torch.device("cuda", 0)
x = torch.zeros(4096, 50, 14, device=dev)
lib = _lib.load()
fn = lib.beast_encode_f32
s = torch.cuda.current_stream(dev).cuda_stream
p = x.data_ptr()
out = {
    "ctypes_encode_B0_19args": t(lambda: fn(p, 0, 50, 700, 14, 1, 14, 14, 14, p, p, 10, p, p, 256, 0, p, p, s)),
    "ctypes_abi_version": t(lambda: lib.beast_abi_version()),
    "current_stream": t(lambda: torch.cuda.current_stream(dev).cuda_stream),
    "raw_stream": t(lambda: torch._C._cuda_getCurrentRawStream(0)),
    "empty_f32": t(lambda: torch.empty((4096, 140), dtype=torch.float32, device=dev)),
    "empty_i64": t(lambda: torch.empty((4096, 140), dtype=torch.int64, device=dev)),
    "to_noop": t(lambda: x.to(dev, dtype=torch.float32)),
    "data_ptr": t(lambda: x.data_ptr()),
    "stride": t(lambda: x.stride()),
    "shape": t(lambda: x.shape),
    "device_eq": t(lambda: x.device == dev),
    "is_cuda_dtype": t(lambda: x.is_cuda and x.dtype is torch.float32),
    "torch_device_ctor": t(lambda: torch.device("cuda:0")),
    "current_device": t(lambda: torch.cuda.current_device()),
    "no_grad_ctx": t(lambda: torch.no_grad().__enter__()),
}
print(json.dumps(out))

# ---- the tokenizer's own path, piece by piece (B=4096, D=14)
from beast_tokenizer_amd import BEASTBsplineTokenizer  # noqa: E402
tok = BEASTBsplineTokenizer(num_dof=14, device="cuda:0")
x = torch.randn(4096, 50, 14, device=dev)
pl = tok._plan()
params = torch.empty((4096, 140), device=dev)
tokens = torch.empty((4096, 140), dtype=torch.int64, device=dev)
xp, pp, tp = x.data_ptr(), params.data_ptr(), tokens.data_ptr()


def enc_call():
    pl.enc(xp, 4096, 50, 700, 14, 1, 14, 14, 14, pl.p_src, pl.p_proj, 10, pl.p_wmn, pl.p_wmx, 256, 0, pp, tp,
           torch._C._cuda_getCurrentRawStream(0))


tok_rows, _ = tok.encode(x)
out2 = {
    "enc_ctypes_plus_launch": t(enc_call, 5000),
    "plan_lookup": t(lambda: tok._plan()),
    "dev_lookup": t(lambda: tok._dev()),
    "fit": t(lambda: tok._fit(x, 0, pl), 5000),
    "encode": t(lambda: tok.encode(x), 5000),
    "fast_encode_only": t(lambda: pl.fast.encode(x, 0, 0), 5000),
    "fast_reconstruct_only": t(lambda: pl.fast.reconstruct(tok_rows, 0, 0), 5000),
    "token_rows": t(lambda: tok._token_rows(tok_rows, pl.dev)),
    "reconstruct_traj": t(lambda: tok.reconstruct_traj(tok_rows), 5000),
}
torch.cuda.synchronize()
print(json.dumps(out2))
