"""One steady-state step of a rocprofv3 kernel trace (csv, optionally
gzipped) between two kernel indices: kernels, busy and wall time, and the
per-kernel totals.  python tools/trace_step.py TRACE FIRST LAST [TOP]
(the step boundaries: the optimizer-chain indices trace_steps.py prints)."""
import gzip, csv, collections, re, sys
op = gzip.open if sys.argv[1].endswith('.gz') else open
rows = list(csv.DictReader(op(sys.argv[1], 'rt')))
rows.sort(key=lambda r: int(r['Start_Timestamp']))
a,b = int(sys.argv[2]), int(sys.argv[3])
step = rows[a:b]
def short(n):
    n=n.replace('(anonymous namespace)::','').replace('void ','').replace('at::native::',''); n=re.sub(r'\(.*','',n)
    n=re.sub(r'std::array<char\*, \d+ul> ','',n)
    return n[:110]
t = collections.Counter(); c = collections.Counter()
for r in step:
    k = short(r['Kernel_Name'])
    if k.startswith('Cijk'): k = 'GEMM ' + k[:40]
    d = (int(r['End_Timestamp'])-int(r['Start_Timestamp']))/1e3
    t[k]+=d; c[k]+=1
wall=(int(step[-1]['End_Timestamp'])-int(step[0]['Start_Timestamp']))/1e3
print(f"kernels {len(step)} busy {sum(t.values())/1e3:.2f} ms wall {wall/1e3:.2f} ms")
for k,v in t.most_common(int(sys.argv[4]) if len(sys.argv)>4 else 50):
    print(f"{v:9.1f} us n={c[k]:4d} avg={v/c[k]:7.1f}  {k}")
