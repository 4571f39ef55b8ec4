#!/bin/bash
# PMC pass (one counter set) per kernel variant on one bench configuration:
#   scripts/pmc_ab.sh "<bench args>" "<label>:<env>" ...
# Output: gpurun_out/pmc_ab/<label>/ (rocprofv3 csv) + summary lines.
set -euo pipefail
export TMPDIR=/tmp
args="$1"; shift
# PMC="<counters>" overrides the default set (at most 8 SQ_ counters per pass).
PMC=${PMC:-"SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_SMEM GRBM_GUI_ACTIVE"}
mkdir -p gpurun_out/pmc_ab
for spec in "$@"; do
  IFS=: read -r label envs <<< "$spec"
  env $envs timeout -s KILL 120 rocprofv3 --pmc $PMC \
    --output-format csv -d gpurun_out/pmc_ab/$label -o run -- python3 bench.py $args > gpurun_out/pmc_ab/$label.json 2> gpurun_out/pmc_ab/$label.err
done
python3 - "$@" <<'PY'
import csv, glob, sys, collections
for spec in sys.argv[1:]:
    label = spec.split(":")[0]
    tot = collections.defaultdict(float); n = 0
    for f in glob.glob(f"gpurun_out/pmc_ab/{label}/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            if "life_" not in r.get("Kernel_Name", ""): continue
            tot[r["Counter_Name"]] += float(r["Counter_Value"])
    v = lambda k: tot.get(k, 0.0)
    print(label, {k: "%.4g" % x for k, x in sorted(tot.items())})
    if v("SQ_WAVES"):
        print("  VALU/wave %.0f  SALU/wave %.0f  VALU per busy cycle %.3f  wait frac %.3f  cycles/wave %.0f" % (
            v("SQ_INSTS_VALU") / v("SQ_WAVES"), v("SQ_INSTS_SALU") / v("SQ_WAVES"),
            v("SQ_ACTIVE_INST_VALU") / max(1, v("SQ_BUSY_CYCLES")), v("SQ_WAIT_INST_ANY") / max(1, v("SQ_WAVE_CYCLES")),
            v("SQ_WAVE_CYCLES") / v("SQ_WAVES")))
PY
