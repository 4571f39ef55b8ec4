#!/bin/bash
# Parallel text I/O at BASELINE sizes (VERDICT r04 "Missing 3"): generate
# 32768^2 and 65536^2 input files, then bin/gol --style collective at 1 rank
# and 8 in-process ranks (1x8, 2x4 on the one GPU), Reading / Writing ms and
# their split (text parse / host->device load, device->host store / text
# format) in --metrics-json, and byte comparisons of the outputs: generation
# 0 against the input itself, 100 generations between the decompositions.
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
O=gpurun_out/${1:-r05/io}
D=${TMPDIR:-/tmp}/gol_io
mkdir -p $O $D
step() {  # step NAME LIMIT CMD...
  local name=$1 limit=$2
  shift 2
  local t0=$SECONDS
  timeout -k 10 "$limit" "$@" > $O/$name.out 2> $O/$name.err
  local rc=$?
  echo "step $name rc=$rc $((SECONDS - t0)) s"
  [ $rc -eq 0 ] || { tail -5 $O/$name.err; exit $rc; }
}
for N in 32768 65536; do
  step gen_$N 300 bin/gol_gen $N $N $D/in_$N.txt 7
  step r1_g0_$N 300 bin/gol $N $N $D/in_$N.txt --style collective --gens 0 --output $D/out_$N.txt --metrics-json $O/r1_g0_$N.json
  step cmp_g0_$N 120 cmp $D/in_$N.txt $D/out_$N.txt
  step r1_g100_$N 300 bin/gol $N $N $D/in_$N.txt --style collective --gens 100 --output $D/o100_$N.txt --metrics-json $O/r1_g100_$N.json
  for d in 1x8 2x4; do
    step r8_${d}_g100_$N 300 bin/gol $N $N $D/in_$N.txt --style collective --gens 100 --ranks 8 --decomp $d --output $D/o100_${d}_$N.txt --metrics-json $O/r8_${d}_g100_$N.json
    step cmp_${d}_$N 120 cmp $D/o100_$N.txt $D/o100_${d}_$N.txt
  done
  rm -f $D/*_$N.txt
done
python3 - "$O" <<'PY'
import glob, json, os, sys
O = sys.argv[1]
print("| run | file GB | Reading ms | parse | load | GB/s read | Writing ms | store | format | GB/s write | Generations | loop ms |")
print("|---|---:|---:|---:|---:|---:|---:|---:|---:|---:|---:|---:|")
for f in sorted(glob.glob(os.path.join(O, "*.json"))):
    d = json.load(open(f)); gb = d["file_bytes"] / 1e9
    print(f"| {os.path.basename(f)[:-5]} | {gb:.2f} | {d['read_ms']:.0f} | {d['read_parse_ms']:.0f} | {d['read_load_ms']:.0f} | "
          f"{gb / (d['read_ms'] / 1e3):.2f} | {d['write_ms']:.0f} | {d['write_store_ms']:.0f} | {d['write_format_ms']:.0f} | "
          f"{gb / (d['write_ms'] / 1e3):.2f} | {d['generations']} | {d['loop_ms']:.1f} |")
PY
