"""Counts the reference traversal work (k-DOP tests without the on-entry re-test,
Moller-Trumbore tests) of each benchmark workload with the oracle's count mode and
writes profiles/work_counts.json (bench.py's algorithmic-byte roofline reads it)."""
import json, os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from raytracercpp_amd import scenes
from oracle.bindings import Oracle

out_path = os.path.join(ROOT, "profiles", "work_counts.json")
data = json.load(open(out_path)) if os.path.exists(out_path) else {}
for name in (sys.argv[1:] or ["sphere1m"]):
    sc, st = scenes.CONFIGS[name]()
    r = Oracle(sc, st).render_rows()
    c = dict(r.counters)
    c["render"] = list(st.render_size())
    c["triangle_sha256"] = sc.triangle_hash()
    c.update({k: v for k, v in data.get(name, {}).items() if k.startswith("pmc_")})
    data[name] = c
    print(name, c)
json.dump(data, open(out_path, "w"), indent=1, sort_keys=True)
