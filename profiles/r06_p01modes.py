#!/usr/bin/env python3
"""Round 6: p = 0.01's detector modes give the same sums -- walk with the LDS filter (the
default before this change), lockstep with the pre-filter and L2 filter (CVD_WALK=0), lockstep
with the whole filter in LDS (CVD_WALK=0 CVD_LDSF_LOCKSTEP=1) -- on a few hundred trials of the
headline's model.  Run as a child per mode (the env is read at model build)."""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CHILD = r'''
import json, sys
sys.path.insert(0, %r)
import __graft_entry__ as g
pkg = g.load_package()
cc = pkg.CONFIG_CODES["m6"]
det = pkg.Detector(1, 2, 6, cc["gen1"], device=0)
m = pkg.Model(det.dec, 0.01, 1_000_000, 200, 1.0, 12345).upload(0)
r = det.run_trials(m, cc["gen1"], cc["gen2"], 20_000, 0.01, 12345, 777, 777 + 640, return_sums=True)
inf = m.info()
print(json.dumps({"walk": inf["walk"], "lds_filter": inf["lds_filter"], "counts": [int(x) for x in (r["counts"].cpu() if hasattr(r["counts"], "cpu") else r["counts"]).tolist()],
                  "sums": (r["sums"].cpu().numpy() if hasattr(r["sums"], "cpu") else r["sums"]).tobytes().hex()}))
''' % ROOT


def main():
    out = {}
    for name, env in (("walk_ldsf", {}), ("lock_pf", {"CVD_WALK": "0"}),
                      ("lock_ldsf", {"CVD_WALK": "0", "CVD_LDSF_LOCKSTEP": "1"})):
        e = dict(os.environ, **env)
        r = subprocess.run([sys.executable, "-c", CHILD], env=e, capture_output=True, text=True, timeout=600)
        if r.returncode:
            print(r.stderr[-3000:])
            sys.exit(1)
        out[name] = json.loads(r.stdout.strip().splitlines()[-1])
    same = len({v["sums"] for v in out.values()}) == 1 and len({str(v["counts"]) for v in out.values()}) == 1
    print(json.dumps({k: {"walk": v["walk"], "lds_filter": v["lds_filter"], "counts": v["counts"]} for k, v in out.items()}))
    print("sums_identical", same)
    sys.exit(0 if same else 1)


if __name__ == "__main__":
    main()
