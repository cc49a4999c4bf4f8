#!/bin/bash
# Phase split of k_thermo_coop on config 4: the tree's library and builds with phases compiled out
# (ab/libdfmi_skip<k>.so, -DDFMI_TSKIP=k: 1 Wilke rows, 2 diffusion pairs, 4 Newton loop), one kernel trace each.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
L=deepflame-dev_amd/libdfmi.so
cp $L /tmp/libdfmi_a.so
for k in ${VARIANTS:-a skip1 skip2 skip4}; do
  case $k in a) cp /tmp/libdfmi_a.so $L ;; *) cp ab/libdfmi_$k.so $L ;; esac
  rm -rf gpurun_out/ts_$k
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/ts_$k -o run -- python3 scripts/config4_profile.py 128 > gpurun_out/ts_$k.log 2>&1
  rc=$?; [ $rc -eq 0 ] || { echo "$k rc=$rc"; cp /tmp/libdfmi_a.so $L; exit $rc; }
  python3 - "$k" <<'PY'
import csv, sys
k = sys.argv[1]
r = [x for x in csv.DictReader(open(f"gpurun_out/ts_{k}/run_kernel_trace.csv")) if "thermo_coop" in x["Kernel_Name"]]
d = [(int(x["End_Timestamp"]) - int(x["Start_Timestamp"])) / 1e3 for x in r]
print(k, [round(v) for v in d])
PY
done
cp /tmp/libdfmi_a.so $L
