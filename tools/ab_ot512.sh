for i in 1 2; do
  timeout -k 10 200 python -u tools/quick_perf.py 20 2>&1 | tail -1 | sed 's/^/default: /'
  FCCF_LIB=fccf-pcr_amd/lib_ot512/libfccf.so FCCF_IS_BLOCK_GRID=496 timeout -k 10 200 python -u tools/quick_perf.py 20 2>&1 | tail -1 | sed 's/^/ot512x2: /'
  FCCF_LIB=fccf-pcr_amd/lib_ot512/libfccf.so timeout -k 10 200 python -u tools/quick_perf.py 20 2>&1 | tail -1 | sed 's/^/ot512x1: /'
done
