# A/B of abl_libs/*.so kernel times without the parity tests (diagnostic builds give wrong results)
KFILT=x bash tools/ab_libs.sh
