# conv32 (fp32 operands) A/B builds under abl_libs/ at cfg4 (profiling), with a bit-identity check of the
# denoiser output against the first library.
set -e
L0=$(ls abl_libs/*.so | head -1)
for L in abl_libs/*.so; do PNP_LIB_PATH=$PWD/$L timeout -k 10 200 python -u tools/c32_bits.py $L.npz; done
for L in abl_libs/*.so; do python -c "import numpy as np; a=np.load('$L0.npz')['y']; b=np.load('$L.npz')['y']; print('$L bit-identical to $L0:', np.array_equal(a, b))"; done
BARGS="--config cfg4 --steps 3" KFILT=x bash tools/ab_libs.sh
