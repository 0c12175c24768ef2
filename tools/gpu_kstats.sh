# kernel time per library variant (rocprofv3 --kernel-trace --stats over tools/ablate.py), one box
# usage: O=gpurun_out/x VARIANTS="libdgj2t libdgj2t_stop1" CFG=c2 bash tools/gpu_kstats.sh
set -o pipefail
O=${O:-gpurun_out/kstats}
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
for rep in ${REPS:-1}; do
for v in ${VARIANTS:-libdgj2t}; do
  DG_ALLOW_STALE=1 DG_LIB_PATH=dynamicgo_amd/$v.so timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $O/${v}_$rep -o run -- python3 tools/ablate.py ${CFG:-c2} > $O/${v}_$rep.log 2>&1 || { tail -20 $O/${v}_$rep.log; exit 1; }
  python3 -c '
import csv,sys
rows=list(csv.DictReader(open(sys.argv[1])))
print(sys.argv[2], " ".join("%s=%.2fus" % (r["Name"].split("(")[0].split("<")[0][-22:], float(r["AverageNs"])/1e3) for r in rows if "j2t" in r["Name"] or "t2j" in r["Name"]))' $O/${v}_$rep/run_kernel_stats.csv $v
done; done
