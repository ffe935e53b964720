#!/bin/bash
# One line per bench log: config, ms/step, pairs/s, dominant-kernel ms and roofline frac.
for f in "$@"; do python3 - "$f" <<'PY'
import json, sys
f = sys.argv[1]
for l in open(f):
    if l.startswith('{"metric'):
        d = json.loads(l); r = d['roofline']
        print("%-40s N=%-5d ms/step %.4f  pairs/s %.3g  kernel %.4f ms  frac %.3f  cand %s" % (
            f.split('/')[-1], d['config']['n_seqs'], d['ms_per_step'], d['value'], r['kernel_ms'], r['frac'],
            r.get('screen', {}).get('candidate_tiles')))
PY
done
