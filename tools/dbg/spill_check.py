"""Debug: records-only routing of the C4 dead25 digest config vs the oracle; where do they differ."""
import json, os, sys
import numpy as np
REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, REPO); sys.path.insert(0, os.path.join(REPO, "oracle"))
import importlib
pkg = importlib.import_module("statsd-router_amd")
import sr_oracle
d = json.load(open(os.path.join(REPO, "tests/golden/digests.json")))
for key in sys.argv[1:]:
    c = d[key]
    s = pkg.gen_stream(c["nbytes"], c["line_lens"], seed=c["seed"], p_invalid=c["p_invalid"])
    words = np.array([int(x, 16) for x in c["alive"]], dtype=np.uint64)
    nd = c["n_downstreams"]
    alive = [int((int(words[k >> 6]) >> (k & 63)) & 1) for k in range(nd)]
    cr, _, cn = sr_oracle.route(s.data, nd, alive)
    with pkg.Router(nd, 16 << 20) as r:
        r.set_alive(words)
        for it in range(2):
            recs, _, n = r.route(s.data)
            bad = np.nonzero(recs != cr)[0]
            print(key, "iter", it, "n", n, cn, "bad", len(bad), flush=True)
            if len(bad):
                offs = cr["offset"][bad]
                tiles = offs // 16384
                print("  first bad", bad[:5], "gpu", recs[bad[:3]], "cpu", cr[bad[:3]], "tiles", np.unique(tiles)[:20], len(np.unique(tiles)), flush=True)
