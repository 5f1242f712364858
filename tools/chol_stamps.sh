#!/bin/bash
# Build the stamped development variant of the library (-DSFM_CHOL_STAMPS:
# s_memrealtime stamps of the Cholesky walker's phases and the helpers'
# publications, compiled into the production source) -> abvar/var_stamps.so
set -e
R=$(cd "$(dirname "$0")/.." && pwd)
V=/tmp/var_stamps
rm -rf $V && mkdir -p $V/sfm_amd && cp -r $R/sfm_amd/csrc $V/sfm_amd/ && rm -rf $V/sfm_amd/csrc/build
ln -sfn $R/include $V/include
mkdir -p $R/abvar
make -s -C $V/sfm_amd/csrc -j8 OUT=$R/abvar/var_stamps.so HIPFLAGS="-O3 -std=c++17 -fPIC --offload-arch=gfx950 -Wall -Wno-unused-function -Wno-unused-value -munsafe-fp-atomics -DSFM_CHOL_STAMPS"
