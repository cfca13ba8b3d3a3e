# A/B timing of libreflow_hip.so builds on the incremental DAG workload
# (configs[2]).  For a gpurun box only: it copies each build over the in-tree
# library of the box's scratch copy, then restores the original.
#   bash tools/dag_ab.sh tools/_var/A.so tools/_var/B.so ...
set -e
lib=reflow_amd/libreflow_hip.so
cp "$lib" /tmp/dag_ab_orig.so
for v in "$@"; do
  cp "$v" "$lib"
  r=$(timeout -k 10 120 python tools/dag_probe.py --dag-steps 50 | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['ms_per_step'], d['mnodes_per_s'])")
  echo "$v: $r"
done
cp /tmp/dag_ab_orig.so "$lib"
