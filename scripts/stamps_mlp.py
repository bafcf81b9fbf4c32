#!/usr/bin/env python3
"""Diagnostic: per-phase s_memtime stamps of the MLP rows kernel (workgroup-lead lane).
Prints the median cycles of each phase over workgroups for a steady-state step."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch

from serverless_learn_amd.data.synthetic import make_mnist_like
from serverless_learn_amd.models.mlp import FusedMLPTrainer
from serverless_learn_amd.ops import _native

B = int(sys.argv[1]) if len(sys.argv) > 1 else 65536
if len(sys.argv) > 2:  # force a rows-kernel tile height (64 / 128 / 256)
    _native.call("sl_mlp_set_rows_bm", int(sys.argv[2]))
x, y = make_mnist_like(B * 2, seed=0)
tr = FusedMLPTrainer(batch=B, device="cuda:0")
tr.load_shard(torch.from_numpy(x), torch.from_numpy(y))
for _ in range(5):
    tr.step()
bm = _native.lib().sl_mlp_rows_bm(B)
S = 20  # stamps per workgroup (ROW_STAMPS in mlp_fused.hip)
st = torch.zeros(B // bm * S, dtype=torch.int64, device="cuda:0")
_native.call("sl_mlp_set_stamps", st.data_ptr())
tr._lc = None; tr._lkey = None
tr.step()
torch.cuda.synchronize()
_native.call("sl_mlp_set_stamps", None)
s = st.view(-1, S)[:, :10].cpu().double()
d = s[:, 1:] - s[:, :-1]
names = ["layer1", "relu1", "layer2+h1", "relu2", "layer3+ce", "dW3 part+dH2", "mask2", "dH1+dh2", "mask1+dh1"]
print(f"B={B} BM={bm} workgroups={s.shape[0]}  total median cycles {float((s[:, 9] - s[:, 0]).median()):.0f}")
for i, n in enumerate(names):
    print(f"  {n:14s} median {float(d[:, i].median()):8.0f}  mean {float(d[:, i].mean()):8.0f}")
e = st.view(-1, S).cpu().double()
if bool((e[:, 12] != 0).all()):
    for n, (i, j) in {"l1 end wait": (1, 12), "relu1 body": (12, 13), "relu1 barrier": (13, 2),
                      "l2 end wait": (3, 14), "relu2+w3 tail": (14, 4), "dH1 mask+bar": (8, 15),
                      "dh1 out+colsum": (15, 9)}.items():
        print(f"  {n:14s} median {float((e[:, j] - e[:, i]).median()):8.0f}")
tot = (s[:, 9] - s[:, 0])
print(f"  WG total cycles: p50 {float(tot.median()):.0f}  p90 {float(tot.quantile(0.9)):.0f}  max {float(tot.max()):.0f}")
# s_memtime counts shader clocks per XCC; s_memrealtime is a 100 MHz clock shared by the whole chip
rt0, rt1 = e[:, 16], e[:, 17]
if bool((rt1 > rt0).all()):
    mhz = tot / ((rt1 - rt0) / 100.0)
    print(f"  shader clock MHz over each WG: median {float(mhz.median()):.0f}  min {float(mhz.min()):.0f}  "
          f"max {float(mhz.max()):.0f}")
    print(f"  start spread (100 MHz clock): median {float((rt0 - rt0.min()).median()) * 10:.0f} ns  "
          f"max {float((rt0 - rt0.min()).max()) * 10:.0f} ns;  first start -> last end "
          f"{float(rt1.max() - rt0.min()) * 10:.0f} ns")

# ---- occupancy reconstruction from placement ids ----
raw = st.view(-1, S).cpu()
hw = raw[:, 10].numpy().astype("int64")
xcc = raw[:, 11].numpy().astype("int64") & 0xF
cu = (hw >> 8) & 0xF
sh = (hw >> 12) & 0x1
se = (hw >> 13) & 0x7
key = xcc * 1000 + se * 100 + sh * 16 + cu
import collections
import numpy as np
t0s = raw[:, 0].numpy().astype("int64")
t1s = raw[:, 9].numpy().astype("int64")
by = collections.defaultdict(list)
for i in range(len(key)):
    by[int(key[i])].append((t0s[i], t1s[i]))
spans, conc, busy = [], [], []
for k, iv in by.items():
    iv.sort()
    lo, hi = min(a for a, _ in iv), max(b for _, b in iv)
    spans.append(hi - lo)
    busy.append(sum(b - a for a, b in iv))
    ev = sorted([(a, 1) for a, _ in iv] + [(b, -1) for _, b in iv])
    c = m = 0
    for _, d in ev:
        c += d
        m = max(m, c)
    conc.append(m)
print(f"CUs seen {len(by)}  WGs/CU median {np.median([len(v) for v in by.values()]):.0f}  "
      f"max concurrency median {np.median(conc):.0f}  span median {np.median(spans):.0f}  "
      f"sum(WG time)/span median {np.median(np.array(busy) / np.array(spans)):.2f}")
xs = collections.Counter(int(x) for x in xcc)
print("WGs per XCC:", dict(sorted(xs.items())))

# ---- the two workgroups sharing a CU: per-phase cycles of the one that ends first vs last ----
dph = s[:, 1:] - s[:, :-1]
first, last, pair_ids = [], [], []
for k, idx in collections.defaultdict(list, {kk: [i for i in range(len(key)) if int(key[i]) == kk]
                                             for kk in set(int(v) for v in key)}).items():
    if len(idx) != 2:
        continue
    i, j = sorted(idx, key=lambda q: t1s[q])
    pair_ids.append((i, j))
    first.append(dph[i].numpy()); last.append(dph[j].numpy())
if first:
    f, l = np.median(np.array(first), 0), np.median(np.array(last), 0)
    print(f"CU pairs {len(first)}: median phase cycles, WG ending first | WG ending last")
    for n_, a_, b_ in zip(names, f, l):
        print(f"  {n_:14s} {a_:8.0f} | {b_:8.0f}")
    half = s.shape[0] // 16  # per XCD: workgroups (blockIdx >> 3) >= half are the younger ones
    young_last = sum(1 for i, j in pair_ids if (j >> 3) >= half)
    mixed = sum(1 for i, j in pair_ids if ((i >> 3) >= half) != ((j >> 3) >= half))
    print(f"  pairs with one older + one younger workgroup: {mixed}/{len(pair_ids)}; "
          f"younger ends last: {young_last}/{len(pair_ids)}")
