"""Writes an instrumented copy of chol_kernels.hip (argv[1] -> argv[2]) with
per-wave clock64 stamps inside potrf_tile, for tools/potrf_tile_micro.hip
(-DCHOL_SRC, -DPOTRF_STAMPS): g_st[wave][id], ids 4b+0 panel start, 4b+1
panel work done, 4b+2 after the barrier, 4b+3 after the trailing update;
16 before the W row 3 finish, 17 at the end."""
import sys
s = open(sys.argv[1]).read()
inc = '#include "/root/repo/sfm_amd/csrc/'
s = s.replace('#include "ba_device.h"', inc + 'ba_device.h"').replace('#include "ba_common.h"', inc + 'ba_common.h"')
decl = ('__device__ long long g_st[4][32];\n'
        '#define STAMP(id) { if ((threadIdx.x & 63) == 0) g_st[threadIdx.x >> 6][id] = clock64(); }\n')
s = s.replace('typedef double f64x4', decl + 'typedef double f64x4', 1)
a = s.index('__device__ __forceinline__ bool potrf_tile(')
e = s.index('  return bad;\n}', a)
body = s[a:e]
body = body.replace('    const int g0 = 16 * b;\n', '    const int g0 = 16 * b;\n    STAMP(4 * b);\n', 1)
body = body.replace('    __syncthreads();\n    // ---- trailing update',
                    '    STAMP(4 * b + 1);\n    __syncthreads();\n    STAMP(4 * b + 2);\n    // ---- trailing update', 1)
body = body.replace('      __syncthreads();\n    }\n  }\n', '      __syncthreads();\n    }\n    STAMP(4 * b + 3);\n  }\n', 1)
body = body.replace('  if (w >= 1) w_row3_finish', '  STAMP(16);\n  if (w >= 1) w_row3_finish', 1)
body = body + '  STAMP(17);\n'
s = s[:a] + body + s[e:]
open(sys.argv[2], 'w').write(s)
