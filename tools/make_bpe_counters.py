"""profiles/r03/bpe_loop_counters.json: the K5 merge loop's per-launch counters (rocprofv3 --pmc,
tools/bpe_pmc.sh, summarised by tools/pmc_summary.py) beside the same kernels' launch durations
(tools/bpe_trace.sh), and what they imply per pass and in HBM bandwidth.

    python tools/make_bpe_counters.py PMC_SUMMARY.json TRACE_SUMMARY.json OUT.json

FETCH_SIZE / WRITE_SIZE are in KiB per launch.  MI355X_MICROARCH.md calibrates FETCH_SIZE at 1/2
of the bytes only for 16-byte-per-lane loads; k_merge_batch's signature scan uses 8-byte loads,
and its FETCH_SIZE agrees with the 38.8 MB signature array (4,850,131 words x 8 B) without the
factor, so the counts are taken as they are."""
import json
import sys

pmc, trace, out = (json.load(open(sys.argv[1])), json.load(open(sys.argv[2])), sys.argv[3])
HBM_PEAK = 8e12
res = {"sources": {"pmc": sys.argv[1], "trace": sys.argv[2]}, "kernels": {}}
for k in ("k_merge_batch", "k_apply_batch"):
    c = pmc.get(k, {})
    t = next((v for n, v in trace["kernels"].items() if n.endswith(k)), None)
    if not c or t is None:
        continue
    rd, wr = c["FETCH_SIZE"] * 1024.0, c["WRITE_SIZE"] * 1024.0
    us = t["mean_us"]
    waves = c.get("SQ_WAVES", 0.0)
    rec = {"launches": t["launches"], "mean_us": us, "fetch_bytes": rd, "write_bytes": wr,
           "hbm_GBps": (rd + wr) / us / 1e3, "hbm_frac": (rd + wr) / (us * 1e-6) / HBM_PEAK}
    if waves:
        rec.update({"waves": waves, "valu_insts_per_wave": c.get("SQ_INSTS_VALU", 0) / waves,
                    "salu_insts_per_wave": c.get("SQ_INSTS_SALU", 0) / waves,
                    "wave_cycles_waiting_frac": c.get("SQ_WAIT_ANY", 0) / c["SQ_WAVE_CYCLES"],
                    "wave_cycles_issuing_frac": c.get("SQ_ACTIVE_INST_ANY", 0) / c["SQ_WAVE_CYCLES"]})
    res["kernels"][k] = rec
m, a = res["kernels"].get("k_merge_batch"), res["kernels"].get("k_apply_batch")
if m and a:
    bytes_pass = m["fetch_bytes"] + m["write_bytes"] + a["fetch_bytes"] + a["write_bytes"]
    res["per_pass"] = {"bytes": bytes_pass, "kernel_us": m["mean_us"] + a["mean_us"],
                       "hbm_GBps_in_kernels": bytes_pass / (m["mean_us"] + a["mean_us"]) / 1e3}
json.dump(res, open(out, "w"), indent=1)
print(json.dumps(res, indent=1))
