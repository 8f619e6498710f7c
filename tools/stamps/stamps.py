"""Phase timeline of workgroup 0 of k_encode / k_reconstruct from in-kernel s_memtime
stamps (a -DBEAST_STAMPS build of csrc/, this tool only; the product compiles them out).

    python tools/stamps/stamps.py [B ...]
"""
import ctypes as C
import glob
import json
import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, REPO)

NW = 8   # stamp slots per kernel (waves per workgroup <= 8 in csrc/codec.hip)
ENC = ["start", "issued", "landed", "mfma_done", "pb_ready", "params_stored", "tokens_stored", "drained", "acc_ready",
       "y_dma", "p_dma", "small_dma", "t2_landed", "t2_mfma_done", "t2_tokens_stored"]
REC = ["start", "issued", "landed", "decoded", "w_ready", "mfma_done", "ob_ready", "stored", "drained",
       "tok_dma", "small_dma", "phi_loads", "lut"]


def build():
    from beast_tokenizer_amd import _build
    so = os.path.join(HERE, "libbeast_stamps.so")
    objs = []
    for src in glob.glob(os.path.join(REPO, "beast_tokenizer_amd", "csrc", "*.hip")):
        o = os.path.join(HERE, os.path.basename(src) + ".o")
        extra = _build.FILE_FLAGS.get(os.path.basename(src), [])
        subprocess.run([_build._hipcc(), *_build.CXXFLAGS, *extra, "-DBEAST_STAMPS", "-c", src, "-o", o], check=True)
        objs.append(o)
    subprocess.run([_build._hipcc(), f"--offload-arch={_build.ARCH}", "-shared", "-o", so, *objs], check=True)
    return so


def grid_of(B):
    return (B + 7) // 8 if "BEAST_DEBUG_GRID_CAP" not in os.environ else min((B + 7) // 8, int(os.environ["BEAST_DEBUG_GRID_CAP"]))


def block_summary(bst, k, nblk):
    """Workgroup lifetimes from s_memrealtime (10 ns ticks): dispatch spread, durations,
    and the spread per XCC (HW_REG_XCC_ID) / CU."""
    import numpy as np
    a = np.array(bst[k * 4096 * 4:(k + 1) * 4096 * 4], dtype=np.uint64).reshape(4096, 4)[:nblk]
    st, en = a[:, 0].astype(np.int64), a[:, 1].astype(np.int64)
    ok = (st > 0) & (en >= st)
    st, en, hw = st[ok], en[ok], a[ok, 2]
    t0 = st.min()
    xcc = (hw >> np.uint64(32)).astype(np.int64) & 0xF
    cu = (hw.astype(np.int64) >> 8) & 0xF
    se = (hw.astype(np.int64) >> 13) & 0x7
    dur = (en - st) * 10
    def q(x):
        return [int(np.percentile(x, p)) for p in (0, 10, 50, 90, 100)]
    out = {"n": int(ok.sum()), "start_ns_pct_0_10_50_90_100": q((st - t0) * 10),
           "end_ns_pct": q((en - t0) * 10), "dur_ns_pct": q(dur),
           "per_xcc_blocks": [int((xcc == x).sum()) for x in range(8)],
           "per_xcc_last_end_ns": [int(((en[xcc == x] - t0) * 10).max()) if (xcc == x).any() else None
                                   for x in range(8)],
           "distinct_cu": int(len(set(zip(xcc.tolist(), se.tolist(), cu.tolist()))))}
    return out


def main():
    import torch
    from beast_tokenizer_amd import BEASTBsplineTokenizer, _lib
    from beast_tokenizer_amd.synthetic import synth_trajectories
    so = os.path.join(HERE, "libbeast_stamps.so")   # built in the container (build()), travels along
    lib = C.CDLL(so if os.path.exists(so) and not os.environ.get("STAMPS_REBUILD") else build())
    for name, (res, args) in _lib.SIGNATURES.items():
        fn = getattr(lib, name)
        fn.restype, fn.argtypes = res, args
    lib.beast_stamps_read.argtypes = [C.c_void_p]
    lib.beast_bstamps_read.argtypes = [C.c_void_p]
    bst = (C.c_ulonglong * (2 * 4096 * 4))()
    dev = torch.device("cuda", 0)
    tok = BEASTBsplineTokenizer(num_dof=14, device="cuda:0")
    p = tok._plan()
    stamps = (C.c_ulonglong * (2 * NW * 16))()
    lib.beast_stamps_read(stamps)
    sizes = [int(v) for v in sys.argv[1:]] or [4096, 1048576]
    if os.environ.get("STAMPS_BLOCKS_ONLY"):
        sizes = sizes
    s = torch._C._cuda_getCurrentRawStream(0)
    out = {}
    for B in sizes:
        x = torch.from_numpy(synth_trajectories(min(B, 65536), 50, 14, seed=0)).to(dev)
        if B > 65536:
            x = x.repeat(B // 65536, 1, 1)
        params = torch.empty((B, 140), device=dev)
        tokens = torch.empty((B, 140), dtype=torch.int64, device=dev)
        pos = torch.empty((B, 50, 14), device=dev)

        def enc():
            return lib.beast_encode_f32(x.data_ptr(), B, 50, 700, 14, 1, 14, 14, 14, p.p_src, p.p_proj, 10, p.p_wmn,
                                        p.p_wmx, 256, 0, params.data_ptr(), tokens.data_ptr(), s)

        def enc_params_only():
            return lib.beast_encode_f32(x.data_ptr(), B, 50, 700, 14, 1, 14, 14, 14, p.p_src, p.p_proj, 10, p.p_wmn,
                                        p.p_wmx, 256, 0, params.data_ptr(), None, s)

        def rec():
            return lib.beast_reconstruct_f32(tokens.data_ptr(), B, 14, 14, 10, 256, 0, p.p_wmn, p.p_wmx, p.p_phi, 0,
                                             50, p.p_dst, 14, None, 0, None, None, pos.data_ptr(), None, s)
        res = {}
        pipe = ["start", "dma_issued", "A_landed", "fitA_done(mw)", "B_landed(mw)", "fitB_done|storeA_done", "bar3",
                "storeB_issued", "drained"]
        for kname, fn, names, k in (("encode", enc, pipe if B <= 8192 else ENC, 0),
                                    ("encode_params_only", enc_params_only, pipe if B <= 8192 else ENC, 0),
                                    ("reconstruct", rec, REC, 1)):
            for _ in range(20):           # warm: code, constants and the tile in L2 as in back-to-back use
                assert fn() == 0
            torch.cuda.synchronize()
            assert lib.beast_stamps_read(stamps) == 0
            v = [stamps[(k * NW + w) * 16: (k * NW + w) * 16 + 16] for w in range(NW)]
            ws = [w for w in range(NW) if v[w][0]]   # waves that stamped (none: kernel without STAMP)
            res[kname] = {}
            if ws:
                t0 = min(v[w][0] for w in ws)
                res[kname] = {names[i]: [int(v[w][i] - t0) if v[w][i] >= t0 else None for w in ws]
                              for i in range(len(names)) if names[i] != "-"}
            assert lib.beast_bstamps_read(bst) == 0
            res[kname]["blocks"] = block_summary(bst, k, min(4096, grid_of(B)))
        out[B] = res
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
