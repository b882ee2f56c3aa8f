"""Where one wave's in-order instruction stream spends its cycles: the
in-order single-wave model of tools/isa_walk.py (issue in program order, each instruction after its
sources are ready; latencies from tools/micro/chain_latency.hip), with every cycle attributed to
issue (by unit), operand stalls (by the producing unit of the latest source) or s_waitcnt waits.

  python tools/inorder_breakdown.py [--k 128 --n 256 --lat profiles/r05d_chain_latency.txt]
"""
import argparse
import collections
import os
import re
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "tools"), os.path.join(ROOT, "tests"), os.path.join(ROOT, "polar-code-pytorch-sionna_amd")]
import isa_walk as w  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--k", type=int, default=128)
ap.add_argument("--n", type=int, default=256)
ap.add_argument("--lat", default=os.path.join(ROOT, "profiles", "r05d_chain_latency.txt"))
a = ap.parse_args()
asm = w.kernel_asm(a.k, a.n, 0)
ins = w.parse(asm)
tr = w.walk(ins)
lat = w.latency_table(a.lat)
ready = {}; t = 0.0; vm, lgkm = [], []
stall = collections.Counter(); issue = collections.Counter(); waitc = collections.Counter(); count = collections.Counter()
producer = {}
for i in tr:
    text = ins[i][1]; m = text.split()[0]
    d, s_ = w.dst_src(text)
    if m == "s_nop":
        n = int(text.split()[1], 0) + 1; t += n; issue['s_nop'] += n; continue
    if m == "s_waitcnt":
        t0 = t
        for part in text.split()[1:]:
            mm = re.match(r"(vmcnt|lgkmcnt)\((\d+)\)", part)
            if mm:
                q = vm if mm.group(1) == "vmcnt" else lgkm
                keep = int(mm.group(2))
                while len(q) > keep:
                    t = max(t, q.pop(0))
                waitc[mm.group(1)] += t - t0; t0 = t
        continue
    lt = w.inst_latency(m, lat)
    srcready = [(ready.get(r, 0.0), r) for r in s_]
    start = max([t] + [x for x, _ in srcready])
    if start > t:
        # attribute the stall to the unit of the producer of the latest source
        r = max(srcready)[1]
        stall[producer.get(r, '?')] += start - t
    done = start + lt
    u = w.unit(m)
    kind = u + ('_dpp' if ('row_' in text or 'quad_perm' in text) else '') + ('_f64' if u == 'valu' and ('f64' in m or 'b64' in m) else '')
    for r in d:
        ready[r] = done; producer[r] = kind
    if u == "vmem" and not m.startswith(("global_store", "buffer_store", "scratch_store")): vm.append(done)
    elif u == "vmem": vm.append(start + 8.0)
    elif u in ("lds", "smem"): lgkm.append(done)
    inc = 1.0 if u in ("salu", "ctl") else 4.0
    issue[kind] += inc; count[kind] += 1
    t = start + inc
end = max([t] + vm + lgkm)
print("in-order cycles", round(end), "instructions", len(tr))
print("issue cycles by kind", {k: round(v) for k, v in issue.most_common()})
print("instruction counts", dict(count.most_common()))
print("operand stalls by producer kind", {k: round(v) for k, v in stall.most_common()})
print("s_waitcnt waits", {k: round(v) for k, v in waitc.items()})
print("tail (outstanding memory after the last issue)", round(end - t))
