#!/bin/bash
# Launch anatomy (tools/anatomy.py) of several library builds under rocprofv3 --kernel-trace, joined
# into gpurun_out/anat_<lib>_<variant>_<mode>_joined.json.  Run on the GPU box:
#   bash tools/anat_ab.sh "base rev" "medium:8 large:16" "tscan default"
# <lib> is build_ab/<lib>.so ("tree" = the in-tree library).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export TMPDIR=/tmp
mkdir -p gpurun_out
for lib in $1; do
  so=build_ab/$lib.so; [ "$lib" = tree ] && so=rllib-warehouse_amd/warehouse/_lib/libwarehouse_amd.so
  for va in $2; do
    v=${va%%:*}; n=${va##*:}
    for mode in $3; do
      tag=${lib}_${v}_${mode}
      extra="--ks 1,2,5,20,100 --reps 3"; [ "$mode" = tscan ] && extra="--tscan --reps 3"
      WAREHOUSE_AMD_LIB=$so timeout -k 10 240 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/anat_$tag -o run \
        -- python3 tools/anatomy.py --variant $v --agents $n $extra > gpurun_out/anat_$tag.json 2> gpurun_out/anat_$tag.err
      rc=$?; echo "$tag rc=$rc"; [ $rc -eq 0 ] || exit $rc
      python3 tools/anatomy.py --join gpurun_out/anat_$tag/run_kernel_trace.csv gpurun_out/anat_$tag.json > gpurun_out/anat_$tag.txt
      rm -f gpurun_out/anat_$tag/run_kernel_trace.csv
    done
  done
done
