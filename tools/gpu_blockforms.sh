#!/bin/bash
# Dev: block-kernel forms.  Ten clouds per launch: the batched sort harness for the
# default library and variants (tools/gpu_sortvar.sh); two clouds (single
# registrations, the 1024-thread form unless FCCF_IS_BLOCK_B2=1): quick_perf.
# Usage (via gpurun): bash tools/gpu_blockforms.sh TAG "sortvar variants" "qp specs"
#   qp spec: lib[:b2]   (lib "base" = lib/, ":b2" sets FCCF_IS_BLOCK_B2=1)
TAG=$1
OUT=gpurun_out/$TAG
mkdir -p $OUT
CHECK=1 bash tools/gpu_sortvar.sh $TAG $2 || exit 1
for r in 1 2; do
  for spec in $3; do
    v=${spec%%:*}
    if [ "$v" = base ]; then L=fccf-pcr_amd/lib/libfccf.so; else L=fccf-pcr_amd/lib_$v/libfccf.so; fi
    E=(FCCF_LIB=$L); [ "$spec" != "$v" ] && E+=(FCCF_IS_BLOCK_B2=1)  # (unset otherwise: "" would select the first form)
    env "${E[@]}" timeout -k 10 120 python -u tools/quick_perf.py > $OUT/qp.txt 2>&1 || { cat $OUT/qp.txt; exit 1; }
    echo "qp $spec: $(tail -1 $OUT/qp.txt)"
  done
done
