#!/bin/bash
# Variant library with the blocked sub-tile TRSM during the panels
# (SFM_CHOL_EXT) -> abvar/var_ext.so; with STAMPS=1 also the stamped build
# -> abvar/var_extst.so
set -e
R=$(cd "$(dirname "$0")/.." && pwd)
F="-O3 -std=c++17 -fPIC --offload-arch=gfx950 -Wall -Wno-unused-function -Wno-unused-value -munsafe-fp-atomics"
for v in ext extst; do
  V=/tmp/var_$v
  rm -rf $V && mkdir -p $V/sfm_amd && cp -r $R/sfm_amd/csrc $V/sfm_amd/ && rm -rf $V/sfm_amd/csrc/build
  ln -sfn $R/include $V/include
  X="-DSFM_CHOL_EXT"; [ $v = extst ] && X="$X -DSFM_CHOL_STAMPS"
  make -s -C $V/sfm_amd/csrc -j8 OUT=$R/abvar/var_$v.so HIPFLAGS="$F $X"
done
