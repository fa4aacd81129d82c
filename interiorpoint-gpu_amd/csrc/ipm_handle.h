// The C-ABI handle (include/ipm355.h: ipm_handle), shared by the translation units that export
// entry points (ipm_engine.hip: Newton path; ipm_lasso.hip: batched ADMM).
#pragma once
#include <hip/hip_runtime.h>

#include <string>

#include "ipm_common.h"

constexpr int IPM_HOST_WORDS = 4096;   // pinned host staging (doubles)

struct ipm_handle {
  int device = 0;
  hipStream_t stream = nullptr;
  bool own_stream = false;
  std::string err;
  double* hbuf = nullptr;  // pinned host staging
  int* dinfo = nullptr;    // device scratch for level-0 potrf
  unsigned* ctl = nullptr; // device control words for level-0 potrs
  double* pws = nullptr;   // device workspace for level-0 potrf (grown on demand)
  int64_t pws_n = 0;
  double* scratch = nullptr;
  size_t scratch_bytes = 0;
  void* rb = nullptr;      // library handle for the least-squares fallback (ipm_lstsq.hip), lazy
  hipEvent_t ev[6];
  double kkt_sum = 0.0, potrf_sum = 0.0;
  int64_t kkt_cnt = 0, potrf_cnt = 0;
  bool timing = false;
  bool kkt_pending = false, potrf_pending = false;
};

#define HIPCHK(h, expr)                                                        \
  do {                                                                         \
    hipError_t _e = (expr);                                                    \
    if (_e != hipSuccess) {                                                    \
      (h)->err = std::string(#expr) + ": " + hipGetErrorString(_e);            \
      return IPM_HIP_ERROR;                                                    \
    }                                                                          \
  } while (0)

// grow-only device scratch owned by the handle (level-0 entry points)
inline double* ipm_handle_scratch(ipm_handle* h, size_t bytes) {
  if (bytes > h->scratch_bytes) {
    if (h->scratch) hipFree(h->scratch);
    h->scratch = nullptr;
    h->scratch_bytes = 0;
    if (hipMalloc((void**)&h->scratch, bytes) != hipSuccess) return nullptr;
    h->scratch_bytes = bytes;
  }
  return h->scratch;
}
