# stamp breakdowns of the diagnostic builds in abl_diag/ (profiling only; ablated builds give wrong results)
for L in abl_diag/*.so; do echo "== $L"; PNP_LIB_PATH=$PWD/$L timeout -k 10 200 python tools/f2_stamps.py || exit 1; done
