set -o pipefail
R=$(pwd)
mkdir -p gpurun_out/paff
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 180 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/paff/ks -o run -- python3 $R/tools/ko_probe.py --steps 4 --warmup 1 --slots 1 > $R/gpurun_out/paff/ks.log 2>&1 || exit 1
timeout -s KILL 180 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU GRBM_GUI_ACTIVE --kernel-trace -d $R/gpurun_out/paff/sq -o run -- python3 $R/tools/ko_probe.py --steps 4 --warmup 1 --slots 1 > $R/gpurun_out/paff/sq.log 2>&1 || exit 1
cd $R
python3 - <<'PY'
import os, sqlite3, glob
def db(d):
    return glob.glob(f"gpurun_out/paff/{d}/**/*results.db", recursive=True)[0]
c = sqlite3.connect(db("ks"))
rows = c.execute("select name, count(*), sum(end-start)/1e3, avg(end-start)/1e3 from kernels group by name order by sum(end-start) desc").fetchall()
out = open("gpurun_out/paff/summary.txt", "w")
for n, k, tot, avg in rows[:25]:
    print(f"{n.split('(')[0][:70]:70s} calls {k:5d} total_us {tot:10.1f} avg_us {avg:9.1f}", file=out)
c = sqlite3.connect(db("sq"))
print("--- counters (per launch avg)", file=out)
for k, n, v in c.execute("select kernel_name, counter_name, avg(value) from counters_collection group by kernel_name, counter_name"):
    if "aff" in k or "accumulate" in k:
        print(f"{k.split('(')[0][:60]:60s} {n:22s} {v:.4g}", file=out)
out.close()
PY
cat gpurun_out/paff/summary.txt
