#!/usr/bin/env python3
"""Run a matrix of bench.py configurations on the GPU box, one process each.

    python scripts/bench_matrix.py MATRIX OUT.jsonl [--repeat N] [--timeout S]

MATRIX lines: ``name | ENV=V ENV2=V2 | bench.py arguments`` (``#`` comments,
blank lines ignored).  Every configuration runs N times, interleaved (all
configurations once, then again), each under its own time limit; each
result line of bench.py is appended to OUT.jsonl with ``name``, ``env`` and
``run`` added.  A run that fails, faults or times out stops the matrix (no
further GPU work in that call) and the exit status says so.  This replaces
the round-specific one-off scripts: profiles/README.md lists which matrix
produced which record."""
from __future__ import annotations

import argparse
import json
import os
import shlex
import subprocess
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def parse(path: str) -> list[tuple[str, dict, list[str]]]:
    rows = []
    for raw in open(path):
        line = raw.split("#", 1)[0].strip()
        if not line:
            continue
        name, env, args = (x.strip() for x in line.split("|"))
        envd = dict(kv.split("=", 1) for kv in shlex.split(env))
        rows.append((name, envd, shlex.split(args)))
    return rows


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("matrix")
    ap.add_argument("out")
    ap.add_argument("--repeat", type=int, default=1)
    ap.add_argument("--timeout", type=int, default=180)
    ap.add_argument("--only", default="", help="comma-separated configuration names to run (default: all)")
    a = ap.parse_args()
    rows = parse(a.matrix)
    if a.only:
        keep = a.only.split(",")
        unknown = sorted(set(keep) - {r[0] for r in rows})
        if unknown:
            print(f"bench_matrix: no configuration named {unknown} in {a.matrix}", file=sys.stderr)
            return 2
        rows = [r for r in rows if r[0] in keep]
    os.makedirs(os.path.dirname(os.path.abspath(a.out)), exist_ok=True)
    log = open(os.path.splitext(a.out)[0] + ".log", "a")
    for run in range(a.repeat):
        for name, env, args in rows:
            cmd = [sys.executable, "-u", os.path.join(REPO, "bench.py"), *args]
            print(f"[{time.strftime('%H:%M:%S')}] run {run} {name}: {' '.join(args)} {env}", flush=True)
            e = dict(os.environ)
            e.update(env)
            t0 = time.time()
            try:
                r = subprocess.run(cmd, env=e, capture_output=True, text=True, timeout=a.timeout, cwd=REPO)
            except subprocess.TimeoutExpired as ex:
                log.write(f"=== {name} run {run}: TIMEOUT after {a.timeout} s\n{ex.stderr or ''}\n")
                log.flush()
                print(f"{name}: timed out; stopping", flush=True)
                return 124
            log.write(f"=== {name} run {run} rc={r.returncode} {time.time() - t0:.1f}s\n{r.stderr[-6000:]}\n")
            log.flush()
            recs = [json.loads(x) for x in r.stdout.splitlines() if x.lstrip().startswith("{")]
            for rec in recs:
                rec.update(name=name, env=env, run=run)
                with open(a.out, "a") as f:
                    f.write(json.dumps(rec) + "\n")
                c = rec.get("config", {})
                print(f"  {name}: {rec['ms_per_step']:.3f} ms/step  {rec['value']:.4g}  verified={rec.get('verified')}"
                      f"  sha={((c.get('verify') or {}).get('final_sha256') or '')[:12]}", flush=True)
            if r.returncode != 0 or not recs:
                print(f"{name}: exit {r.returncode}; stopping (see {log.name})", flush=True)
                print(r.stderr[-3000:], flush=True)
                return r.returncode or 1
    return 0


if __name__ == "__main__":
    raise SystemExit(main())
