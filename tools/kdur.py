"""Median kernel durations from a rocprofv3 kernel trace directory."""
import collections
import csv
import glob
import statistics
import sys

KEYS = ('k_ms_fused_w1', 'k_ms_mask_fast', 'k_ms_select_fast', 'k_ms_decode_fast', 'k_mt_jump', 'k_mt_gen', 'k_mt_seq',
        'k_randk_gather', 'k_decode_scatter1', 'k_qsgd_encode', 'k_absmax', 'k_qsgd_decode', 'k_lane_pack')
dur = collections.defaultdict(list)
for p in glob.glob(f'{sys.argv[1]}/**/*kernel_trace.csv', recursive=True):
    for r in csv.DictReader(open(p)):
        for k in KEYS:
            if k in r['Kernel_Name']:
                name = k + ('<1>' if k == 'k_mt_gen' and 'k_mt_gen<1>' in r['Kernel_Name'] else '')
                dur[name].append((int(r['End_Timestamp']) - int(r['Start_Timestamp'])) / 1e3)
for k, v in dur.items():
    print(f'{k:20s} {statistics.median(v):8.1f} us  ({len(v)})')
