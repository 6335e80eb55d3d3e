"""Per-role kernel times from rocprofv3 rocpd SQLite databases of the DiT loop (diagnostic; the .db form of
tools/trace_split.py): the attention and the N = K = 3072 gated-residual GEMM launch twice per block (self / cross,
proj / cross-proj); split by launch order. Usage: python tools/trace_split_db.py run_results.db ..."""
import sqlite3
import statistics as st
import sys

for f in sys.argv[1:]:
    c = sqlite3.connect(f)
    cols = [r[1] for r in c.execute("pragma table_info(kernels)")]
    ts = "start" if "start" in cols else [x for x in cols if "start" in x][0]
    rows = list(c.execute(f"select name, duration, {ts} from kernels order by {ts}"))

    def durs(sub):
        return [d / 1e3 for n, d, s in rows if sub in n]

    att = durs("attn_fwd_hd256")
    pr = durs("gemm_bf16_kernel<2, false, 7>")
    cq = durs("gemm_bf16_kernel<5, false, 7>")
    print(f.split("/")[-2], "self", round(st.mean(att[0::2]), 1), "cross", round(st.mean(att[1::2]), 1),
          "proj", round(st.mean(pr[0::2]), 1), "cproj", round(st.mean(pr[1::2]), 1), "crossq", round(st.mean(cq), 1),
          "n", len(att), len(pr))
