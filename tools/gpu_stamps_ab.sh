set -e
for L in ${LIBS}; do echo "== $L"; PNP_LIB_PATH=$PWD/abl_libs/$L.so timeout -k 10 120 python -u tools/stack_stamps.py; done
