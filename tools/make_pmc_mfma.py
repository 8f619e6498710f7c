"""profiles/pmc_mfma.json from rocprofv3 --pmc passes of tools/pmc_codec.py (tools/gpu_pmc.sh):
per-launch MFMA instruction counts of the fit kernel, the input of bench.py's ``mfma`` object.

    python tools/make_pmc_mfma.py gpurun_out/mfma_4096 gpurun_out/mfma_262144 [out.json]

Each root holds one pass of SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_SALU
(kernel-trace only) at the batch named by the directory suffix.  SQ_INSTS_MFMA counts wave-level
MFMA instructions; every one in k_encode is v_mfma_f32_16x16x4_f32 = 16*16*4*2 = 2048 flops.
"""
import json
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
from pmc_summary import summarise  # noqa: E402

roots = [a for a in sys.argv[1:] if os.path.isdir(a)]
out = next((a for a in sys.argv[1:] if a.endswith(".json")),
           os.path.join(os.path.dirname(HERE), "profiles", "pmc_mfma.json"))
res = {"method": "rocprofv3 --pmc SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_SALU --kernel-trace "
                 "over tools/pmc_codec.py (50 launches per kernel), mean per dispatch",
       "flops_per_mfma": 2048, "sources": [os.path.basename(r.rstrip("/")) for r in roots], "launches": {}}
for r in roots:
    B = int(r.rstrip("/").rsplit("_", 1)[1])
    s = summarise(r)
    for k in ("k_encode", "k_reconstruct"):
        c = s.get(k)
        if not c:
            continue
        res["launches"][f"{k.split('_', 1)[1]}_{B}"] = {
            "kernel": k, "batch": B, "mfma_insts_per_launch": c.get("SQ_INSTS_MFMA"),
            "mfma_busy_cycles_per_launch": c.get("SQ_VALU_MFMA_BUSY_CYCLES"),
            "valu_insts_per_launch": c.get("SQ_INSTS_VALU"), "salu_insts_per_launch": c.get("SQ_INSTS_SALU")}
json.dump(res, open(out, "w"), indent=1)
print(json.dumps(res, indent=1))
