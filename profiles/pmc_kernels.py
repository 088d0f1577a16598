#!/usr/bin/env python3
"""Per-kernel PMC table from several rocprofv3 --pmc pass directories (each with a counter_collection
CSV): the average per dispatch of every counter, kernels ordered by their summed duration in the first
pass's kernel trace.   python3 profiles/pmc_kernels.py DIR1 [DIR2 ...]"""
import csv
import glob
import os
import re
import sys
from collections import defaultdict


def short(n):
    return re.sub(r'\(.*$', '', re.sub(r'^void\s+', '', n)).replace('cnf::', '').strip()


per = defaultdict(lambda: defaultdict(list))
dur = defaultdict(float)
for i, d in enumerate(sys.argv[1:]):
    for f in glob.glob(os.path.join(d, '**', '*counter_collection.csv'), recursive=True):
        for r in csv.DictReader(open(f)):
            per[short(r['Kernel_Name'])][r['Counter_Name']].append(float(r['Counter_Value']))
    if i == 0:
        for f in glob.glob(os.path.join(d, '**', '*kernel_trace.csv'), recursive=True):
            for r in csv.DictReader(open(f)):
                dur[short(r['Kernel_Name'])] += (int(r['End_Timestamp']) - int(r['Start_Timestamp'])) / 1e3
for k in sorted(per, key=lambda k: -dur.get(k, 0))[:16]:
    c = {n: sum(v) / len(v) for n, v in per[k].items()}
    wc = c.get('SQ_WAVE_CYCLES', 0) or 1
    parts = [f"{k[:34]:34s} {dur.get(k, 0):9.1f}us"]
    if 'SQ_WAVE_CYCLES' in c:
        parts.append(f"waves {c.get('SQ_WAVES', 0):7.0f} wait {c.get('SQ_WAIT_ANY', 0) / wc:4.2f} "
                     f"stall {c.get('SQ_WAIT_INST_ANY', 0) / wc:4.2f} active {c.get('SQ_ACTIVE_INST_ANY', 0) / wc:4.2f} "
                     f"mfma {c.get('SQ_INSTS_MFMA', 0):9.0f} valu {c.get('SQ_INSTS_VALU', 0):9.0f}")
    if 'SQ_INSTS_LDS' in c:
        parts.append(f"lds {c['SQ_INSTS_LDS']:8.0f} conf {c.get('SQ_LDS_BANK_CONFLICT', 0):8.0f} "
                     f"ldsact {c.get('SQ_LDS_IDX_ACTIVE', 0):9.0f} ldsstall {c.get('SQ_WAIT_INST_LDS', 0):9.0f}")
    if 'FETCH_SIZE' in c:
        parts.append(f"fetch {2 * c['FETCH_SIZE'] / 1024:8.2f} MB")
    if 'WRITE_SIZE' in c:
        parts.append(f"write {c['WRITE_SIZE'] / 1024:8.2f} MB")
    print(' | '.join(parts))
