// Internal seam between the KLT handle (klt_kernels.hip) and the corner
// detector (gftt_kernels.hip): the detector runs on the handle's current
// frame (level 0, resident in HBM) and keeps its device state in the handle.
#pragma once
#include <hip/hip_runtime.h>
#include <cstdint>
#include "../../include/sfm_amd.h"

struct KltFrame {
  const uint8_t* img;  // current frame, level 0, [h][w] u8 (device)
  int w, h;
  hipStream_t stream;
  void** gftt_slot;    // detector state owned by the handle
};

// 0, or SFM_EINVAL when no frame has been pushed.
int sfm_internal_klt_frame(sfm_klt_handle* h, KltFrame* out);
// Frees a detector state (called from sfm_klt_destroy).
void sfm_internal_gftt_free(void* state);
