"""Fold a profile directory's per-run bench JSON lines into one file (profiles hygiene).

Each ``*.json`` file under DIR holding JSON (one object, or JSON lines) is appended to
``DIR/runs.jsonl`` as ``{"file": <path relative to DIR>, "data": <object>}`` and removed; READMEs,
CSV kernel traces, logs and text summaries stay.  The numbers the DESIGN cites stay readable in
one file per directory instead of hundreds.  Usage: python tools/consolidate_profiles.py DIR...
(profiles/traffic and profiles/mfma are read by bench.py at run time: never pass them)."""

import json
import os
import sys


def consolidate(d):
    if os.path.basename(os.path.normpath(d)) in ("traffic", "mfma"):
        raise SystemExit("%s is read by bench.py" % d)
    out = os.path.join(d, "runs.jsonl")
    rows = []
    if os.path.exists(out):
        rows = [json.loads(l) for l in open(out) if l.strip()]
    done = []
    for root, _, files in os.walk(d):
        for f in sorted(files):
            if not f.endswith(".json"):
                continue
            p = os.path.join(root, f)
            text = open(p).read().strip()
            try:
                objs = [json.loads(text)]
            except ValueError:
                try:
                    objs = [json.loads(l) for l in text.splitlines() if l.strip()]
                except ValueError:
                    continue   # not JSON: leave the file
            for o in objs:
                rows.append({"file": os.path.relpath(p, d), "data": o})
            done.append(p)
    if not done:
        return 0
    with open(out, "w") as fh:
        for r in rows:
            fh.write(json.dumps(r, sort_keys=True) + "\n")
    for p in done:
        os.remove(p)
    for root, dirs, files in sorted(os.walk(d, topdown=False)):
        if root != d and not os.listdir(root):
            os.rmdir(root)
    return len(done)


if __name__ == "__main__":
    for d in sys.argv[1:]:
        print(d, consolidate(d))
