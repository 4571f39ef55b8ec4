#!/usr/bin/env python3
"""Run bench.py over a list of configurations and collect the JSON lines.

Each configuration is one line of the spec file: optional VAR=value
environment assignments followed by bench.py arguments, e.g.

    GOL_MIN_SEG_ROWS=128 --tmax 8 --layout u8

Stops at the first failing configuration (a failed GPU step ends the run).
"""
import json
import os
import shlex
import subprocess
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def main() -> int:
    spec, out = sys.argv[1], sys.argv[2]
    timeout = int(os.environ.get("SWEEP_TIMEOUT", "240"))
    with open(out, "w") as f:
        for line in open(spec):
            line = line.strip()
            if not line or line.startswith("#"):
                continue
            toks = shlex.split(line)
            env = dict(os.environ)
            args = []
            for t in toks:
                if "=" in t and not t.startswith("-") and not args:
                    k, v = t.split("=", 1)
                    env[k] = v
                else:
                    args.append(t)
            t0 = time.time()
            r = subprocess.run(["timeout", "-k", "10", str(timeout), sys.executable, os.path.join(REPO, "bench.py"),
                                *args], env=env, capture_output=True, text=True)
            if r.returncode != 0:
                print(f"FAILED ({r.returncode}): {line}\n{r.stderr[-2000:]}", file=sys.stderr, flush=True)
                return 1
            rec = json.loads([ln for ln in r.stdout.splitlines() if ln.startswith("{")][-1])
            rec["sweep_config"] = line
            tune = [ln for ln in r.stderr.splitlines() if "autotune" in ln]
            if tune:
                rec["autotune_log"] = tune[:64]
            rec["wall_s"] = round(time.time() - t0, 2)
            f.write(json.dumps(rec) + "\n")
            f.flush()
            gps = rec.get("config", {}).get("gens_per_step", 1)
            print(f"{rec['value']:.4e}  {rec['ms_per_step'] * 1e3 / gps:8.3f} us/gen  {line}", flush=True)
    return 0


if __name__ == "__main__":
    raise SystemExit(main())
