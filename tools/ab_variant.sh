#!/bin/bash
mkdir -p gpurun_out/ab2
timeout -k 5 120 python -u tools/quick_perf.py > gpurun_out/ab2/base1.log 2>&1 || exit 1
FCCF_LIB=fccf-pcr_amd/lib_ot512/libfccf.so timeout -k 5 120 python -u tools/quick_perf.py > gpurun_out/ab2/ot512_1.log 2>&1 || exit 1
timeout -k 5 120 python -u tools/quick_perf.py > gpurun_out/ab2/base2.log 2>&1 || exit 1
FCCF_LIB=fccf-pcr_amd/lib_ot512/libfccf.so timeout -k 5 120 python -u tools/quick_perf.py > gpurun_out/ab2/ot512_2.log 2>&1 || exit 1
FCCF_LIB=fccf-pcr_amd/lib_ot512/libfccf.so timeout -k 5 300 python -u -m pytest tests/test_gpu_introsort.py tests/test_gpu_register.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/ab2/ot512_tests.log 2>&1
echo "tests rc=$?"
for f in gpurun_out/ab2/*.log; do echo "$f: $(tail -1 $f)"; done
