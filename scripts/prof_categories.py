#!/usr/bin/env python
"""Group a rocprofv3 *_kernel_stats.csv by op class (ms per unit)."""
import collections
import csv
import sys


def cat_of(n):
    if 'igemm_fwd' in n or 'conv_fwd' in n: return 'conv_fwd(miopen)'
    if 'igemm_bwd' in n or 'bwd_data' in n: return 'conv_bwd_data(miopen)'
    if 'igemm_wrw' in n or 'bwd_weight' in n or 'wrw' in n: return 'conv_wrw(miopen)'
    if 'rs::' in n: return 'ours:' + n.split('(')[0].split('<')[0].replace('void ', '')
    if 'SubTensorOp' in n or 'OpTensor' in n: return 'miopen_tensorop(bias)'
    if 'batch_norm' in n or 'BatchNorm' in n: return 'bn'
    if 'reduce_kernel' in n: return 'reduce(sum)'
    if 'Cijk' in n: return 'hipblaslt_gemm'
    if 'copy' in n.lower() or 'fill' in n.lower(): return 'copy/fill'
    if 'elementwise' in n: return 'elementwise'
    if 'Cat' in n: return 'cat'
    return 'other:' + n[:70]


def main(path, div=1.0):
    cat = collections.Counter(); calls = collections.Counter()
    for r in csv.DictReader(open(path)):
        c = cat_of(r['Name'])
        cat[c] += float(r['TotalDurationNs']) / 1e6 / div
        calls[c] += int(r['Calls']) / div
    tot = sum(cat.values())
    print(f"{path}: total {tot:.2f} ms/unit")
    for k, v in cat.most_common(40):
        print(f"  {v:8.3f} ms {100 * v / tot:5.1f}%  {calls[k]:7.0f} calls  {k}")


if __name__ == '__main__':
    main(sys.argv[1], float(sys.argv[2]) if len(sys.argv) > 2 else 1.0)
