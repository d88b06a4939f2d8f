"""Summary of tools/chain_pmc.sh: the SQ counters of the timed k_chain3 launch (the second
chain dispatch of the microbenchmark), per SGD step and per wave, beside the static census.
    python tools/chain_pmc_summary.py gpurun_out/chain_pmc base > profiles/r02_chain_pmc.json"""
import collections
import csv
import json
import sys

root, tag = sys.argv[1], sys.argv[2] if len(sys.argv) > 2 else "base"
STEPS = 400 * 2 * 4           # updates x epochs x minibatches (tools/chain_pmc.sh: 400 updates)
out = {"source": f"tools/chain_pmc.sh {tag} (rocprofv3 --pmc, 2 passes of 8 SQ counters, "
                 "tools/bin/bench_chain_<tag>_<net> 400 updates, one chain workgroup = 4 waves)",
       "units": "SQ_*_CYCLES / SQ_WAIT_* / SQ_ACTIVE_INST_* in quad-cycles (x4 = shader cycles, "
                "MI355X_MICROARCH.md), per SGD step per wave; SQ_INSTS_* per SGD step per wave"}
for net in ("br", "ar"):
    tot = collections.defaultdict(float)
    for p in (1, 2):
        rows = list(csv.DictReader(open(f"{root}/{tag}_{net}_p{p}/pmc_counter_collection.csv")))
        chain = sorted({int(r["Dispatch_Id"]) for r in rows if "k_chain3" in r["Kernel_Name"]})
        for r in rows:
            if int(r["Dispatch_Id"]) == chain[-1]:
                tot[r["Counter_Name"]] += float(r["Counter_Value"])
    waves = tot["SQ_WAVES"]
    per = {k: v / STEPS / waves for k, v in tot.items() if k != "SQ_WAVES"}
    wc = per["SQ_WAVE_CYCLES"]
    out[net] = {"waves": waves, "per_step_per_wave": per,
                "shader_cycles_per_step": 4 * wc,
                "frac_active_inst": per["SQ_ACTIVE_INST_ANY"] / wc,
                "frac_wait_any (s_waitcnt / barrier parked)": per["SQ_WAIT_ANY"] / wc,
                "frac_wait_inst_any (issue stall)": per["SQ_WAIT_INST_ANY"] / wc,
                "insts_per_step": {k[9:]: per[k] for k in per if k.startswith("SQ_INSTS_")}}
print(json.dumps(out, indent=1))
