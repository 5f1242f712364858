// Two-view triangulation of new map points (the GeometryUtils::
// triangulatePoints call of CSfM::mapping, /root/reference/CSfM.cpp:156, and
// of the initialisation, :918), restated as cv::triangulatePoints (OpenCV
// 3.0 cvTriangulatePoints) on the projection matrices K[R|t]: per point the
// 4x4 system  x P_3 - P_1,  y P_3 - P_2  of both views, its right singular
// vector of the smallest singular value (cv::SVD, cv_linalg.h), then the
// homogeneous division.  GeometryUtils lives in the absent cvUtils library,
// so the K[R|t] composition is the build's reading (parity unpinned; oracle:
// oracle/pnp_oracle.py triangulate_points).  One lane per point.
#include <hip/hip_runtime.h>
#include <map>
#include <string>
#include "../../include/sfm_amd.h"
#include "cv_linalg.h"

void sfm_internal_set_error(const std::string& msg);

namespace sfm {
namespace {

// x = [R|t] X then K x, as P = K [R|t] (3x4, row-major) per camera
__global__ __launch_bounds__(256) void k_triangulate(int n, const int32_t* __restrict__ cam0,
                                                     const int32_t* __restrict__ cam1, const double* __restrict__ uv0,
                                                     const double* __restrict__ uv1, const double* __restrict__ P,
                                                     double* __restrict__ X, double* __restrict__ w4) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const double* Pa = P + 12 * size_t(cam0[i]);
  const double* Pb = P + 12 * size_t(cam1[i]);
  double A[4][4];
  const double xa = uv0[2 * i], ya = uv0[2 * i + 1], xb = uv1[2 * i], yb = uv1[2 * i + 1];
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    A[0][k] = xa * Pa[8 + k] - Pa[k];
    A[1][k] = ya * Pa[8 + k] - Pa[4 + k];
    A[2][k] = xb * Pb[8 + k] - Pb[k];
    A[3][k] = yb * Pb[8 + k] - Pb[4 + k];
  }
  double U[4][4], w[4], Vt[4][4];
  cv_svd<4, 4>(A, U, w, Vt);
  const double h = Vt[3][3];
  X[3 * size_t(i)] = Vt[3][0] / h;
  X[3 * size_t(i) + 1] = Vt[3][1] / h;
  X[3 * size_t(i) + 2] = Vt[3][2] / h;
  if (w4) w4[i] = h;
}

// Per calling thread and device: a stream and a grow-only buffer, kept
// between calls (triangulation runs once per keyframe pair in the mapping
// loop: creating a stream and allocating per call cost ~4 ms per call).
struct TriCtx {
  hipStream_t s = nullptr;
  char* buf = nullptr;
  size_t cap = 0;
};
struct TriCache {
  std::map<int, TriCtx> by_dev;
  ~TriCache() {
    for (auto& kv : by_dev) {
      (void)hipSetDevice(kv.first);
      if (kv.second.s) (void)hipStreamDestroy(kv.second.s);
      if (kv.second.buf) (void)hipFree(kv.second.buf);
    }
  }
};
TriCtx* tri_ctx(int device, size_t bytes) {
  static thread_local TriCache cache;
  TriCtx& c = cache.by_dev[device];
  if (!c.s && hipStreamCreateWithFlags(&c.s, hipStreamNonBlocking) != hipSuccess) {
    c.s = nullptr;
    return nullptr;
  }
  if (c.cap < bytes) {
    if (c.buf) (void)hipFree(c.buf);
    c.buf = nullptr;
    c.cap = 0;
    if (hipMalloc(&c.buf, bytes) != hipSuccess) return nullptr;
    c.cap = bytes;
  }
  return &c;
}

}  // namespace
}  // namespace sfm

using namespace sfm;

extern "C" int sfm_triangulate_points(int32_t device, int32_t n, const int32_t* cam0, const int32_t* cam1,
                                      const double* uv0, const double* uv1, int32_t n_cams, const double* P,
                                      double* X) {
  auto fail = [](int code, const char* m) {
    sfm_internal_set_error(m);
    return code;
  };
  if (n < 0 || n_cams < 0) return fail(SFM_EINVAL, "negative size");
  if (n == 0) return 0;
  if (!cam0 || !cam1 || !uv0 || !uv1 || !P || !X) return fail(SFM_EINVAL, "NULL argument");
  for (int32_t i = 0; i < n; ++i)
    if (cam0[i] < 0 || cam0[i] >= n_cams || cam1[i] < 0 || cam1[i] >= n_cams)
      return fail(SFM_EINVAL, "camera index out of range");
  int ndev = 0;
  if (hipGetDeviceCount(&ndev) != hipSuccess || device < 0 || device >= ndev) return fail(SFM_ENODEV, "no device");
  if (hipSetDevice(device) != hipSuccess) return fail(SFM_ENODEV, "hipSetDevice failed");
  // one buffer for inputs and output (keyframe-sized batches), kept per thread
  const size_t b_idx = sizeof(int32_t) * 2 * size_t(n), b_uv = sizeof(double) * 4 * size_t(n),
               b_P = sizeof(double) * 12 * size_t(n_cams), b_X = sizeof(double) * 3 * size_t(n);
  TriCtx* ctx = tri_ctx(device, b_idx + b_uv + b_P + b_X + 64);
  if (!ctx) return fail(SFM_ENOMEM, "stream or device buffer allocation failed");
  char* buf = ctx->buf;
  int32_t* d_c = reinterpret_cast<int32_t*>(buf);
  double* d_uv = reinterpret_cast<double*>(buf + ((b_idx + 15) & ~size_t(15)));
  double* d_P = d_uv + 4 * size_t(n);
  double* d_X = d_P + 12 * size_t(n_cams);
  hipStream_t s = ctx->s;
  int rc = 0;
  if (hipMemcpyAsync(d_c, cam0, sizeof(int32_t) * n, hipMemcpyHostToDevice, s) != hipSuccess ||
      hipMemcpyAsync(d_c + n, cam1, sizeof(int32_t) * n, hipMemcpyHostToDevice, s) != hipSuccess ||
      hipMemcpyAsync(d_uv, uv0, sizeof(double) * 2 * n, hipMemcpyHostToDevice, s) != hipSuccess ||
      hipMemcpyAsync(d_uv + 2 * size_t(n), uv1, sizeof(double) * 2 * n, hipMemcpyHostToDevice, s) != hipSuccess ||
      hipMemcpyAsync(d_P, P, b_P, hipMemcpyHostToDevice, s) != hipSuccess)
    rc = fail(SFM_EIO, "upload failed");
  if (!rc) {
    k_triangulate<<<(n + 255) / 256, 256, 0, s>>>(n, d_c, d_c + n, d_uv, d_uv + 2 * size_t(n), d_P, d_X, nullptr);
    if (hipMemcpyAsync(X, d_X, b_X, hipMemcpyDeviceToHost, s) != hipSuccess || hipStreamSynchronize(s) != hipSuccess)
      rc = fail(SFM_EIO, "triangulation failed");
  }
  return rc;
}
