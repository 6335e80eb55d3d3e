"""Per-role kernel times from a rocprofv3 --kernel-trace CSV of the DiT loop (diagnostic): the attention and the
N = K = 3072 gated-residual GEMM launch twice per block (self / cross, proj / cross-proj), which --stats averages
together; this splits them by launch order. Usage: python tools/trace_split.py run_kernel_trace.csv ..."""
import csv, sys, statistics as st
def load(f):
    rows = list(csv.DictReader(open(f)))
    rows.sort(key=lambda r: int(r['Start_Timestamp']))
    return rows
for f in sys.argv[1:]:
    rows = load(f)
    def durs(sub):
        return [(int(r['End_Timestamp']) - int(r['Start_Timestamp'])) / 1e3 for r in rows if sub in r['Kernel_Name']]
    att = durs('attn_fwd_hd256'); pr = durs('gemm_bf16_kernel<2, false, 7>'); cq = durs('gemm_bf16_kernel<5, false, 7>')
    print(f.split('/')[-2], 'self', round(st.mean(att[0::2]), 1), 'cross', round(st.mean(att[1::2]), 1),
          'proj', round(st.mean(pr[0::2]), 1), 'cproj', round(st.mean(pr[1::2]), 1), 'crossq', round(st.mean(cq), 1),
          'n', len(att), len(pr))
