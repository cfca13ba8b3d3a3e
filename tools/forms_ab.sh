# A/B of libreflow_hip.so builds with tools/dag_forms.py (for a gpurun box:
# copies each build over the in-tree library of the box's scratch copy, then
# restores the original).
#   bash tools/forms_ab.sh "<dag_forms args>" tools/_var/A.so tools/_var/B.so ...
set -e
args=$1; shift
lib=reflow_amd/libreflow_hip.so
cp "$lib" /tmp/forms_ab_orig.so
for v in "$@"; do
  cp "$v" "$lib"
  echo "== $v"
  timeout -k 10 300 python tools/dag_forms.py $args 2>&1 >/dev/null | grep "ms/step"
done
cp /tmp/forms_ab_orig.so "$lib"
