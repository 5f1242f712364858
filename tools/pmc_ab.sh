#!/bin/bash
# FETCH_SIZE / WRITE_SIZE (separate --pmc passes, MI355X_MICROARCH.md "HBM")
# of the kernels matching $1 on one C3 solve (tools/pmc_c3.py solve), under
# the library variants abvar/var_<name>.so given as the other arguments.
set -o pipefail
R=$GRAFT_REPO_ROOT
RX=$1; shift
cd /tmp && export TMPDIR=/tmp
for v in "$@"; do
  OUT=$R/gpurun_out/pmcab_$v
  rm -rf $OUT && mkdir -p $OUT
  for ctr in FETCH_SIZE WRITE_SIZE "TCC_HIT_sum TCC_MISS_sum"; do
    name=$(echo $ctr | cut -d' ' -f1)
    SFM_AMD_LIB=$R/abvar/var_$v.so timeout -s KILL 120 rocprofv3 --pmc $ctr --kernel-include-regex "$RX" --output-format csv -d $OUT/$name -- python3 $R/tools/pmc_c3.py solve > $OUT/$name.log 2>&1 || exit 1
  done
  echo "== $v"; python3 $R/tools/pmcsum.py $OUT
done
