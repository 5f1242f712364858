#!/bin/bash
# Build an ablation variant: tools/mkvar.sh NAME 'python patch' [file] -> abvar/var_NAME.so (git-ignored; delete after the A/B so it stops shipping)
# The patch is python code run with s = the file's text (default ba_kernels.hip); it must change s.
set -e
R=$(cd "$(dirname "$0")/.." && pwd)
name=$1; patch=$2; file=${3:-ba_kernels.hip}
V=/tmp/var_$name
rm -rf $V && mkdir -p $V/sfm_amd && cp -r $R/sfm_amd/csrc $V/sfm_amd/ && rm -rf $V/sfm_amd/csrc/build
ln -s $R/include $V/include
python3 - "$patch" $V/sfm_amd/csrc/$file <<'PY'
import sys
code, path = sys.argv[1], sys.argv[2]
s = open(path).read(); s0 = s
exec(code)
assert s != s0, "patch changed nothing"
open(path, 'w').write(s)
PY
make -s -C $V/sfm_amd/csrc -j8 OUT=$R/abvar/var_$name.so
