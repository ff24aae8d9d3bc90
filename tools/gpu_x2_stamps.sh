set -e
PNP_LIB_PATH=$PWD/abl_libs/stk_stamps.so timeout -k 10 120 python -u tools/stack_stamps.py 4
PNP_LIB_PATH=$PWD/abl_libs/stk_stamps.so timeout -k 10 120 python -u tools/stack_stamps.py 3
