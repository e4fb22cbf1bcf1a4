"""Per-kernel summary of one rocprofv3 SQ counter pass (tools/pmc_sq.sh):
parked = SQ_WAIT_ANY / SQ_WAVE_CYCLES (waves waiting on s_waitcnt / barriers),
issue-stalled = SQ_WAIT_INST_ANY / SQ_WAVE_CYCLES, active = SQ_ACTIVE_INST_ANY /
SQ_WAVE_CYCLES, LDS bank conflicts = SQ_LDS_BANK_CONFLICT / SQ_LDS_IDX_ACTIVE.
    python tools/pmc_sq.py <counter_collection.csv>  -> JSON on stdout"""
import csv
import json
import sys
from collections import defaultdict


def main():
    acc = defaultdict(lambda: defaultdict(float))
    n = defaultdict(set)
    with open(sys.argv[1]) as fh:
        for row in csv.DictReader(fh):
            k = row["Kernel_Name"].replace("(anonymous namespace)::", "").split("(")[0].replace("void ", "").strip()
            acc[k][row["Counter_Name"]] += float(row["Counter_Value"])
            n[k].add(row.get("Dispatch_Id", ""))
    out = {"source": "rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS "
                      "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VALU (one pass), 1-stream bench", "kernels": {}}
    for k, c in sorted(acc.items(), key=lambda kv: -kv[1].get("SQ_WAVE_CYCLES", 0)):
        wc = c.get("SQ_WAVE_CYCLES", 0)
        if wc <= 0:
            continue
        lds = c.get("SQ_LDS_IDX_ACTIVE", 0)
        out["kernels"][k] = {
            "dispatches": len(n[k]),
            "parked": round(c.get("SQ_WAIT_ANY", 0) / wc, 3),
            "issue_stalled": round(c.get("SQ_WAIT_INST_ANY", 0) / wc, 3),
            "active": round(c.get("SQ_ACTIVE_INST_ANY", 0) / wc, 3),
            "lds_wait": round(c.get("SQ_WAIT_INST_LDS", 0) / wc, 3),
            "lds_bank_conflict_frac": round(c.get("SQ_LDS_BANK_CONFLICT", 0) / lds, 3) if lds else None,
            "valu_insts": c.get("SQ_INSTS_VALU", 0),
        }
    json.dump(out, sys.stdout, indent=1)


if __name__ == "__main__":
    main()
