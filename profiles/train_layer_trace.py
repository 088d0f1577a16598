#!/usr/bin/env python3
"""Per-dispatch view of one coupling layer's training backward (cnf_coupling_backward) at a bench
batch: run under `rocprofv3 --kernel-trace --output-format csv` and fold with --fold.

    rocprofv3 --kernel-trace --output-format csv -d OUT -o run -- python3 tools/train_layer_trace.py cfg2 64 2
    python3 tools/train_layer_trace.py --fold OUT
"""
import csv
import glob
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def run(name, B, layer_ci, reps=3):
    import numpy as np
    import torch
    from arl_conditional_normalizing_flows_amd.config import PRESETS
    from arl_conditional_normalizing_flows_amd.make_model import cFlow
    cfg = PRESETS[name]
    flow = cFlow(**cfg.kwargs(), device=torch.device('cuda', 0), seed=0)
    layers = [L for L in flow.layers_list if hasattr(L, 'coupling_index')]
    L = layers[layer_ci]
    rng = np.random.default_rng(0)
    shp = (B, L.input_height, L.input_width, L.input_depth)
    u = torch.from_numpy(rng.standard_normal(shp).astype(np.float32)).cuda()
    dv = torch.from_numpy(rng.standard_normal(shp).astype(np.float32)).cuda()
    for _ in range(reps):
        L.gradients(u, dv, -1.0 / B)
        torch.cuda.synchronize()
        torch.cuda._sleep(50_000_000)
        torch.cuda.synchronize()
    print(f'{name} B={B} coupling {layer_ci}: {shp}')


def fold(out):
    files = glob.glob(os.path.join(out, '**', '*kernel_trace.csv'), recursive=True)
    rows = []
    for f in files:
        with open(f) as fh:
            rows += list(csv.DictReader(fh))
    rows.sort(key=lambda r: int(r['Start_Timestamp']))
    # reps are separated by torch's GPU sleep kernel (at::cuda::...): keep the last rep
    reps = [[]]
    for r in rows:
        if 'at::' in r['Kernel_Name']:
            reps.append([])
        else:
            reps[-1].append(r)
    rows = [x for x in reps if x][-1]
    t0 = int(rows[0]['Start_Timestamp'])
    tend = max(int(r['End_Timestamp']) for r in rows)
    busy = {}
    for r in rows:
        nm = r['Kernel_Name'].split('(')[0].replace('void ', '').replace('cnf::', '')
        d = (int(r['End_Timestamp']) - int(r['Start_Timestamp'])) / 1e3
        g = f"{r.get('Grid_Size_X', r.get('Grid_Size', ''))}x{r.get('Grid_Size_Y', '')}x{r.get('Grid_Size_Z', '')}"
        print(f"{(int(r['Start_Timestamp']) - t0) / 1e3:9.1f} {d:8.1f} us q{r.get('Queue_Id', '?'):>3} {nm:40s} grid {g} lds {r.get('LDS_Block_Size', r.get('Lds_Size', ''))}")
        busy[nm] = busy.get(nm, 0.0) + d
    print(f'span {(tend - t0) / 1e3:.1f} us, kernel sum {sum(busy.values()):.1f} us')
    for k, v in sorted(busy.items(), key=lambda kv: -kv[1]):
        print(f'  {k:40s} {v:9.1f} us')


if __name__ == '__main__':
    if sys.argv[1] == '--fold':
        fold(sys.argv[2])
    else:
        run(sys.argv[1], int(sys.argv[2]), int(sys.argv[3]))
