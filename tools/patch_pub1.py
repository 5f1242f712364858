# Patch for tools/mkvar.sh (file chol_kernels.hip): waves 1-3 drain and flag
# L_j,j-1 in phase 1 instead of at the start of phase 0 (A/B variant).
def _rep(s, old, new):
    assert s.count(old) == 1, "patch_pub1: anchor not found:\n" + old
    return s.replace(old, new)
blk = '''      if (io.pub_flag != nullptr) {
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        // every lane adds (lane 0 one, the rest zero): the count is uniform
        const int old = __builtin_amdgcn_readfirstlane(atomicAdd(io.pub_cnt, (t & 63) == 0 ? 1 : 0));
        if (old == 2) {  // the third of waves 1-3
          *io.pub_cnt = 0;
          __hip_atomic_store(io.pub_flag, io.epoch, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
      }
'''
s = _rep(s, blk, '')
s = _rep(s, '''      // panel 0's trailing update of blocks (2,2) (3,2) (3,3) [waves 1, 2, 3]
      trail_block(T, 0, w == 1 ? 2 : 3, w == 3 ? 3 : 2, lane);''', blk + '''      // panel 0's trailing update of blocks (2,2) (3,2) (3,3) [waves 1, 2, 3]
      trail_block(T, 0, w == 1 ? 2 : 3, w == 3 ? 3 : 2, lane);''')
