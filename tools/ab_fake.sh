for lib in ${LIBS:-main fake}; do
  if [ $lib = main ]; then L=pquic_amd/lib/libpquic_fec.so; else L=pquic_amd/lib/variants/$lib/libpquic_fec.so; fi
  export PQUIC_AMD_LIB=$PWD/$L
  echo "== $lib"
  timeout -k 10 120 python tools/kernel_only.py enc 16 4 1048576 5 || exit 1
  timeout -k 10 120 python tools/kernel_only.py enc 32 8 1048576 5 || exit 1
  FEC_L=9000 timeout -k 10 120 python tools/kernel_only.py enc 64 16 65536 5 || exit 1
done
