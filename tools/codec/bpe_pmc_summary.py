"""Summarise tools/codec/bpe_encode_pmc.sh's rocprofv3 databases for k_bpe_encode (tools only).
    python tools/codec/bpe_pmc_summary.py gpurun_out/bpe_pmc > profiles/r02/bpe_encode_pmc.json
"""
import json
import os
import sqlite3
import sys


def main(d):
    out = {"kernel": "k_bpe_encode<true>", "workload": "4,096 rows x 140 bins, K5 model (vocab 2,048, 1,724 merges)"}
    c = sqlite3.connect(os.path.join(d, "trace", "run_results.db"))
    n, avg = c.execute("select count(*), avg(end-start) from kernels where name like '%k_bpe_encode%'").fetchone()
    out["launches"], out["avg_duration_ns"] = n, avg
    cnt = {}
    for p in ("p1", "p2"):
        c = sqlite3.connect(os.path.join(d, p, "run_results.db"))
        for name, s, k in c.execute("select counter_name, sum(counter_value), count(distinct dispatch_id) from pmc_events "
                                    "where name like '%k_bpe_encode%' group by counter_name"):
            cnt[name] = s / k   # summed over the counter's instances, per launch
    out["counters_per_launch"] = cnt
    waves = cnt["SQ_WAVES"]
    out["per_wave"] = {k: cnt[k] / waves for k in ("SQ_INSTS_VALU", "SQ_INSTS_SALU", "SQ_INSTS_LDS", "SQ_INSTS_VMEM",
                                                   "SQ_INSTS_SMEM")}
    wc = cnt["SQ_WAVE_CYCLES"]
    out["wave_cycle_split"] = {"parked (SQ_WAIT_ANY)": cnt["SQ_WAIT_ANY"] / wc,
                               "issuing (SQ_ACTIVE_INST_ANY)": cnt["SQ_ACTIVE_INST_ANY"] / wc,
                               "issue stall (SQ_WAIT_INST_ANY)": cnt["SQ_WAIT_INST_ANY"] / wc}
    out["lds_bank_conflict_cycles_over_lds_active"] = cnt["SQ_LDS_BANK_CONFLICT"] / cnt["SQ_ACTIVE_INST_LDS"]
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main(sys.argv[1])
