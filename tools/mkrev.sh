#!/bin/bash
# Build the library of an earlier git revision: tools/mkrev.sh NAME REV -> abvar/var_NAME.so
set -e
R=$(cd "$(dirname "$0")/.." && pwd)
name=$1; rev=$2
V=/tmp/rev_$name
rm -rf $V && mkdir -p $V
git -C $R archive $rev sfm_amd/csrc include | tar -x -C $V
make -s -C $V/sfm_amd/csrc -j8 OUT=$R/abvar/var_$name.so
