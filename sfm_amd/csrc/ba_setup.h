// Launchers of the device-side problem setup (ba_setup.hip), driven by
// sfm_ba_set_problem (ba_solver.hip).
#pragma once
#include <hip/hip_runtime.h>
#include <cstddef>
#include <cstdint>

namespace sfm {

// Temporary-storage bytes of the hipcub primitives for n items: which = 64 /
// 32 (radix sort of uint64 / uint32 keys with int32 values), 1 / 2
// (exclusive sum of int32 / int64).
size_t setup_sort_bytes(int64_t n, int which);
hipError_t sort_pairs64(void* tmp, size_t bytes, const uint64_t* kin, uint64_t* kout, const int32_t* vin,
                        int32_t* vout, int64_t n, uint64_t max_key, hipStream_t s);
hipError_t sort_pairs32(void* tmp, size_t bytes, const uint32_t* kin, uint32_t* kout, const int32_t* vin,
                        int32_t* vout, int64_t n, uint64_t max_key, hipStream_t s);
hipError_t exclusive_sum32(void* tmp, size_t bytes, const int32_t* in, int32_t* out, int64_t n, hipStream_t s);
hipError_t exclusive_sum64(void* tmp, size_t bytes, const int64_t* in, int64_t* out, int64_t n, hipStream_t s);

// Several 32-bit fills in one launch (set_problem's initialisations: one
// kernel instead of one hipMemset each).
struct Fill32Set {
  struct Job { uint32_t* p; int64_t n; uint32_t v; } job[8];
  int n = 0;
  void add(void* p, size_t bytes, uint32_t v) { job[n++] = Job{static_cast<uint32_t*>(p), int64_t(bytes / 4), v}; }
};
void launch_fill32(const Fill32Set& fs, hipStream_t s);
// small device -> pinned host copies (dst: device-mapped pointers of pinned
// host memory; 4-B words) by one kernel, not by the copy engine
struct HostCopySet {
  int n = 0;
  int32_t* dst[4];
  const int32_t* src[4];
  int words[4];
  void add(void* d, const void* s, size_t bytes) {
    dst[n] = static_cast<int32_t*>(d);
    src[n] = static_cast<const int32_t*>(s);
    words[n] = int(bytes / 4);
    ++n;
  }
};
void launch_copy_to_host(const HostCopySet& cs, hipStream_t s);
// pinned host bytes (a device-mapped pointer; bytes a multiple of 16) copied
// by a kernel on s, not by the copy engine
void launch_copy_from_host(void* dst, const void* src_host_mapped, size_t bytes, hipStream_t s);

// err[0..2] = first observation with a bad camera index / point index /
// non-finite uv (INT32_MAX: none); per-camera and per-point counts of the
// observations with valid indices.
void launch_validate(int64_t N, const double* uv, const int32_t* cam, const int32_t* pt, int C, int P, int32_t* err,
                     int32_t* cam_cnt, int32_t* pt_cnt, hipStream_t s);
void launch_pm_keys(int64_t N, const int32_t* cam, const int32_t* pt, int C, uint64_t* keys, int32_t* iota,
                    hipStream_t s);
void launch_gather_pm(int64_t N, const int32_t* order, const double* uv, const int32_t* cam, const int32_t* pt,
                      double* uv_pm, int32_t* cam_pm, int32_t* pt_s, uint32_t* cam_key, int32_t* iota, hipStream_t s);
void launch_fill_cm(int64_t N_pad, const int32_t* wcam, const int32_t* cam_rng, const int32_t* cam_off,
                    const int32_t* cm_order, const int32_t* pt_s, const double* uv_pm, int32_t* cm_p, double* uv_cm,
                    int32_t* cam_obs, int32_t* pos, hipStream_t s);
// (set_problem's deferred uv: uv_pm and uv_cm from the caller-order uv once
// it has landed, k_gather_pm / k_fill_cm having run with uv = nullptr)
void launch_uv_layout(int64_t N, int64_t N_pad, const int32_t* order, const int32_t* wcam, const int32_t* cam_rng,
                      const int32_t* cam_off, const int32_t* cm_order, const double* uv, double* uv_pm, double* uv_cm,
                      int32_t* err, hipStream_t s);
// pt_off (P + 1 entries) from the sorted point-major keys point * C + camera
void launch_pt_off(int P, const uint64_t* sorted_keys, int64_t N, int C, int32_t* pt_off, hipStream_t s);
void launch_chunk_keys(int n, const int4* ch, const int32_t* cm_order, const int32_t* pt_s, int P, uint32_t* key,
                       int32_t* iota, hipStream_t s);
void launch_chunk_gather(int n, const int32_t* perm, const int4* ch, const uint32_t* key, int4* out, int32_t* grp,
                         hipStream_t s);
// cnt[i] (i < N) = pairs of camera-major list entry i; cnt[N] = 0
void launch_pair_count(int64_t N, const int32_t* cm_order, const int32_t* cam_pm, const int32_t* pt_s,
                       const int32_t* pt_off, int64_t* cnt, hipStream_t s);
void launch_pair_fill(int64_t N, const int32_t* cm_order, const int32_t* cam_pm, const int32_t* pt_s,
                      const int32_t* pt_off, const int64_t* off, int C, uint32_t* key, int32_t* val, hipStream_t s);
void launch_seg(int64_t n_blk, const uint32_t* key, int64_t n_pairs, int32_t* seg, hipStream_t s);
void launch_blk(int C, int2* blk, hipStream_t s);
// Keyframe-sized problems: the same layouts without radix sorts (scatter into
// the host-known point segments then ranks within each, per-camera stable
// compactions, run lengths of the camera-sorted point segments for the pair
// lists).  fill / tmp: zeroed point counters (P) and N-item scratch.  Bounds
// (the host checks): C <= 256, at most kSmallChunks chunks, short point
// segments.
constexpr int kSmallSetupMaxC = 256;
constexpr int kSmallSetupMaxChunks = 2048;
constexpr int kSmallSetupMaxPtObs = 64;
constexpr int64_t kSmallSetupMaxObs = 64 * 1024;  // (k_small_cm_compact: 64 steps of 1024)
void launch_small_pm(int64_t N, const int32_t* pt, const int32_t* cam, const double* uv, const int32_t* pt_off,
                     int32_t* fill, int32_t* tmp, int32_t* order, double* uv_pm, int32_t* cam_pm, int32_t* pt_s,
                     hipStream_t s);
void launch_small_cm(int64_t N, int C, const int32_t* cam_pm, const int32_t* cam_off, int32_t* cm_order,
                     hipStream_t s);
void launch_small_chunks(int n, const int4* ch, const int32_t* cm_order, const int32_t* pt_s, int P, int4* out,
                         int32_t* grp, hipStream_t s);
// cnt (n_blk) per block, seg (n_blk + 1) their exclusive sum
void launch_small_pairs_count(int C, int64_t n_blk, const int32_t* cam_off, const int32_t* cm_order,
                              const int32_t* cam_pm, const int32_t* pt_s, const int32_t* pt_off, int32_t* cnt,
                              int32_t* seg, hipStream_t s);
void launch_small_pairs_fill(int C, int64_t n_blk, const int32_t* cam_off, const int32_t* cm_order,
                             const int32_t* cam_pm, const int32_t* pt_s, const int32_t* pt_off, const int32_t* seg,
                             int32_t* bpts, hipStream_t s);
// k_schur_pts work order (XCD-aware, set_problem step 5): bperm (room for
// bperm_slots_bound slots) gets every block in its slot, -1 elsewhere; grp
// [16] = each group's first block and block count (the launch's grid is
// max_x ceil(count_x / per) * 8 workgroups).  key_a / key_b / iota / sorted
// hold n_blk items, row_x C; sort_tmp as setup_sort_bytes(n_blk, 32).
int64_t bperm_slots_bound(int64_t n_blk, int per);
hipError_t launch_bperm(int C, int64_t n_blk, int64_t n_pairs, const int32_t* seg, const int2* blk, int per,
                        uint32_t* key_a, uint32_t* key_b, int32_t* iota, int32_t* sorted, int32_t* row_x,
                        int64_t* grp, void* sort_tmp, size_t sort_bytes, int32_t* bperm, hipStream_t s);

}  // namespace sfm
