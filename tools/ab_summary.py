import json, sys
for l in open(sys.argv[1] if len(sys.argv) > 1 else 'gpurun_out/ab.log'):
    v, js = l.split(' ', 1)
    d = json.loads(js)
    k = d['kernels']
    print(f"{v:22s} {d['ms_per_step']:8.1f} ms  " + " ".join(f"{n[:8]} {k[n]['ms_per_step']:7.1f}" for n in ('lstm_fwd_step', 'lstm_bwd_step', 'gcn_layer', 'wgrad', 'dx', 'head_loss')))
