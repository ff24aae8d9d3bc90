# Build an A/B variant of libpnppds.so into abl_libs/<name>.so with extra -D flags on one source
# (SRCF=ops default, or conv) (profiling only; the product library is pnp-pds_amd/lib).
#   bash tools/build_ab.sh <name> -DX=1 ...
set -e
N=$1; shift
make -C pnp-pds_amd -j8 > /dev/null
mkdir -p abl_libs/$N.obj
S=${SRCF:-ops}
F=${SRCFILE:-csrc/$S.hip}   # SRCFILE: another version of that source (absolute path), e.g. from git show
(cd pnp-pds_amd && /opt/rocm/bin/hipcc -O3 -std=c++17 --offload-arch=gfx950 -fPIC -mllvm -pragma-unroll-threshold=200000 -I csrc "$@" -c $F -o ../abl_libs/$N.obj/$S.o)
O=$(ls pnp-pds_amd/build/*.o | grep -v "/$S.o")
/opt/rocm/bin/hipcc -O3 -std=c++17 --offload-arch=gfx950 -fPIC -shared -o abl_libs/$N.so abl_libs/$N.obj/$S.o $O
rm -rf abl_libs/$N.obj
echo built abl_libs/$N.so
