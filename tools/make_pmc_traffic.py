"""profiles/pmc_traffic.json from rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes
(tools/gpu_pmc.sh over tools/pmc_codec.py at the bench's batch).

HBM bytes per launch = 2 * FETCH_SIZE + WRITE_SIZE, both KiB -> bytes.  The factor 2 is
the gfx950 correction of MI355X_MICROARCH.md (FETCH_SIZE reports half the bytes of a
wide coalesced read, 16 B/lane -- the DMA and vector loads here are all 16 B/lane);
WRITE_SIZE is exact for 16-B-per-lane stores.
    python tools/make_pmc_traffic.py gpurun_out/pmc_4096 [out.json]
"""
import json
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
from pmc_summary import summarise  # noqa: E402

root = sys.argv[1]
out = sys.argv[2] if len(sys.argv) > 2 else os.path.join(os.path.dirname(HERE), "profiles", "pmc_traffic.json")
s = summarise(root)
res = {"source": os.path.basename(root.rstrip("/")), "batch": 4096,
       "method": "rocprofv3 --pmc FETCH_SIZE (own pass) and WRITE_SIZE (own pass), --kernel-trace; "
                 "bytes = 2 * FETCH_SIZE[KiB] * 1024 + WRITE_SIZE[KiB] * 1024 (gfx950 FETCH_SIZE half-count)"}
for k, c in s.items():
    fetch = 2 * c.get("FETCH_SIZE", 0.0) * 1024
    write = c.get("WRITE_SIZE", 0.0) * 1024
    res[k] = {"fetch_bytes_per_launch": fetch, "write_bytes_per_launch": write,
              "hbm_bytes_per_launch": fetch + write}
json.dump(res, open(out, "w"), indent=1)
print(json.dumps(res, indent=1))
