// Error plumbing and identification for libhiseg.
#include <hip/hip_runtime.h>
#include <stdarg.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <atomic>
#include "hiseg.h"
#include "hiseg_data.h"
#include "hiseg_distill.h"
#include "hiseg_head_train.h"
#include "hiseg_loss.h"
#include "hiseg_train.h"

static thread_local char g_err[512] = "";

void hiseg_set_error(const char* fmt, ...) {
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(g_err, sizeof(g_err), fmt, ap);
  va_end(ap);
}

int hiseg_check_launch(const char* what) {
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) {
    hiseg_set_error("%s: launch failed: %s", what, hipGetErrorString(e));
    return HISEG_ERR_LAUNCH;
  }
  return HISEG_OK;
}

static std::atomic<long long> g_place_declined{0}, g_place_far{0};

// Diagnostic: HISEG_LOG_PLACEMENT=1 reports every kernel choice that depended on where two operands lie in memory;
// hiseg_placement_stats counts them ("... declined ..." notes: a fallback kernel took the layer).
void hiseg_note_placement(const char* what, const hiseg_conv2d_desc* d) {
  (strstr(what, "declined") ? g_place_declined : g_place_far).fetch_add(1);
  static const bool on = getenv("HISEG_LOG_PLACEMENT") != nullptr;
  if (on)
    fprintf(stderr, "[hiseg placement] %s: A %p (%d ch) B %p (%d ch) -> %d, %dx%d taps, N %d %dx%d, convT %d up %d\n",
            what, d->srcA, d->Ca, d->srcB, d->Cb, d->Cout, d->KH, d->KW, d->N, d->H, d->W, d->convT, d->a_up);
}

// Diagnostic: HISEG_PLACEMENT_FAR=1 makes every two-source layer take the path of sources lying far apart.
bool hiseg_force_far() {
  static const bool on = getenv("HISEG_PLACEMENT_FAR") != nullptr;
  return on;
}

extern "C" int hiseg_placement_stats(long long* declined, long long* far, int reset) {
  if (declined) *declined = g_place_declined.load();
  if (far) *far = g_place_far.load();
  if (reset) {
    g_place_declined = 0;
    g_place_far = 0;
  }
  return HISEG_OK;
}

extern "C" int hiseg_struct_sizes(long long* out, int n) {
  const long long sz[] = {(long long)sizeof(hiseg_roi_align_desc), (long long)sizeof(hiseg_conv2d_desc),
                          (long long)sizeof(hiseg_wgrad_map),      (long long)sizeof(hiseg_pack_entry),
                          (long long)sizeof(hiseg_bn_apply_desc),  (long long)sizeof(hiseg_bn_bwd_desc),
                          (long long)sizeof(hiseg_ln_bwd_desc),    (long long)sizeof(hiseg_ew_view),
                          (long long)sizeof(hiseg_ubf_desc),       (long long)sizeof(hiseg_ubf_grads),
                          (long long)sizeof(hiseg_loss_cfg),       (long long)sizeof(hiseg_distill_cfg),
                          (long long)sizeof(hiseg_roi_target_desc)};
  const int m = (int)(sizeof(sz) / sizeof(sz[0]));
  for (int i = 0; i < n && i < m; ++i) out[i] = sz[i];
  return m;
}

extern "C" int hiseg_version(void) { return 100; }
extern "C" const char* hiseg_last_error_string(void) { return g_err; }
extern "C" int hiseg_built_for_gfx950(void) { return 1; }

extern "C" int hiseg_stream_create_cu_mask(const unsigned* mask, int nwords, hiseg_stream_t* out) {
  if (!mask || nwords <= 0 || !out) {
    hiseg_set_error("stream_create_cu_mask: bad args");
    return HISEG_ERR_BAD_ARG;
  }
  hipStream_t s = nullptr;
  const hipError_t e = hipExtStreamCreateWithCUMask(&s, (uint32_t)nwords, mask);
  if (e != hipSuccess) {
    hiseg_set_error("stream_create_cu_mask: %s", hipGetErrorString(e));
    return HISEG_ERR_LAUNCH;
  }
  *out = (hiseg_stream_t)s;
  return HISEG_OK;
}

extern "C" int hiseg_stream_destroy(hiseg_stream_t s) {
  const hipError_t e = hipStreamDestroy((hipStream_t)s);
  if (e != hipSuccess) {
    hiseg_set_error("stream_destroy: %s", hipGetErrorString(e));
    return HISEG_ERR_LAUNCH;
  }
  return HISEG_OK;
}
