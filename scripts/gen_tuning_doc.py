#!/usr/bin/env python3
"""Regenerate docs/TUNING.md from the native tuning table (csrc/src/tuning.cpp).

    python scripts/gen_tuning_doc.py
"""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)

from gol_amd._native import native  # noqa: E402

CLASSES = {"tune": "Performance knobs of the default build",
           "diag": "Traces, logs and consistency checks",
           "fault": "Fault injection (tests)",
           "emul": "CPU backend emulating device features (tests)"}


def main() -> None:
    keys = native().tuning_keys()
    out = ["# Runtime tuning keys", "",
           "Generated from the tuning table (`csrc/src/tuning.cpp`; `bin/gol --tune help` prints the same;",
           "regenerate with `python scripts/gen_tuning_doc.py`). Set a key with `--tune key=value` (bin/gol,",
           "`python -m gol_amd.cli`, bench.py) or `LifeConfig(tune={key: value})`; its `GOL_*` variable",
           "overrides the default (precedence: default < environment < explicit). Backends, the engine and",
           "the transports read the table once, at construction. The kernel variants and schedules measured",
           "slower than the defaults were removed in round 6 (their numbers: docs/HISTORY.md).", ""]
    for c, title in CLASSES.items():
        out += [f"## {c}: {title}", "", "| key | environment | default | meaning |", "|---|---|---|---|"]
        for k in keys:
            if k["class"] == c:
                d = k["default"] or "''"
                out.append(f"| `{k['key']}` | `{k['env']}` | `{d}` | {k['doc'].replace('|', '/')} |")
        out.append("")
    with open(os.path.join(REPO, "docs", "TUNING.md"), "w") as f:
        f.write("\n".join(out))


if __name__ == "__main__":
    main()
