"""Summarise an A/B log (lines '<lib> <bench json>'): ms per meta-step and per kernel category."""
import json
import sys

CATS = ('gcn_layer', 'lstm_fwd_step', 'lstm_fwd_dual', 'lstm_bwd_step', 'lstm_bwd_dual', 'wgrad', 'wgrad_reduce')
for line in open(sys.argv[1] if len(sys.argv) > 1 else 'gpurun_out/ab.log'):
    v, js = line.split(' ', 1)
    d = json.loads(js)
    k = d['kernels']
    print(f"{v:26s} {d['ms_per_step']:8.1f} ms  " +
          " ".join(f"{n.replace('lstm_', '')[:9]} {k[n]['ms_per_step']:6.1f}" for n in CATS if n in k))
