// eao_accel.cpp -- C ABI of the engine (include/eao_accel.h). Host glue only:
// argument checks, staging of host buffers, launches on the handle's stream.
// There is deliberately no CPU compute path: without a gfx950 device every
// entry point fails with EAO_E_NODEVICE.
#include "../../include/eao_accel.h"

#include <hip/hip_runtime.h>

#include <cstring>
#include <memory>
#include <string>

#include "assoc.h"
#include "common.h"
#include "hsa_lane.h"
#include "match.h"
#include "orb.h"

namespace eao {
static thread_local std::string g_err;
void set_error(const std::string& s) { g_err = s; }
}  // namespace eao

using namespace eao;

struct eao_orb {
  OrbEngine e;
};

extern "C" {

const char* eao_version(void) { return "eao-slam-amd 0.1 (gfx950)"; }
const char* eao_last_error(void) { return g_err.c_str(); }

int eao_device_ok(int device) {
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess || device < 0 || device >= n) return 0;
  hipDeviceProp_t prop;
  if (hipGetDeviceProperties(&prop, device) != hipSuccess) return 0;
  return std::strncmp(prop.gcnArchName, "gfx950", 6) == 0 ? 1 : 0;
}

static int need_device(int device) {
  if (!eao_device_ok(device)) {
    set_error("no usable gfx950 device (the engine has no CPU fallback)");
    return EAO_E_NODEVICE;
  }
  return EAO_OK;
}

int eao_lane_selftest(int device, int* out1) {
  if (int rc = need_device(device)) return rc;
  if (hipSetDevice(device) != hipSuccess) return EAO_E_HIP;
  if (!eao::hsa_lanes_available(device)) {
    set_error("eao_lane_selftest: HSA lanes unavailable on this device (or EAO_HSA_LANES=0)");
    return EAO_E_STATE;
  }
  return eao::lane_selftest(device, out1);
}

int eao_orb_create(const eao_orb_params* p, int device, eao_orb** out) {
  if (!p || !out) return EAO_E_ARG;
  *out = nullptr;
  int rc = need_device(device);
  if (rc) return rc;
  std::unique_ptr<eao_orb> h(new eao_orb());
  rc = h->e.init(*p, device);
  if (rc) return rc;
  *out = h.release();
  return EAO_OK;
}

int eao_orb_destroy(eao_orb* h) {
  delete h;
  return EAO_OK;
}

int eao_orb_scale_tables(const eao_orb* h, float* scale, float* inv_scale, float* sigma2,
                         float* inv_sigma2) {
  if (!h) return EAO_E_ARG;
  for (int i = 0; i < h->e.p.nlevels; i++) {
    if (scale) scale[i] = h->e.scale[i];
    if (inv_scale) inv_scale[i] = h->e.inv_scale[i];
    if (sigma2) sigma2[i] = h->e.sigma2[i];
    if (inv_sigma2) inv_sigma2[i] = h->e.inv_sigma2[i];
  }
  return EAO_OK;
}

int eao_orb_level_quotas(const eao_orb* h, int32_t* q) {
  if (!h || !q) return EAO_E_ARG;
  for (int i = 0; i < h->e.p.nlevels; i++) q[i] = h->e.quotas[i];
  return EAO_OK;
}

int eao_orb_frame_capacity(const eao_orb* h) { return h ? h->e.cap : EAO_E_ARG; }

int eao_orb_extract(eao_orb* h, const uint8_t* gray, int w, int hh, int stride, eao_keypoint* kps,
                    uint8_t* desc, int cap, int* n_out) {
  if (!h || !n_out) return EAO_E_ARG;
  *n_out = 0;
  if (!gray || w <= 0 || hh <= 0) return EAO_OK;  // _image.empty() -> return
  OrbEngine& e = h->e;
  if (w != e.p.width || hh != e.p.height || stride < w) {
    set_error("eao_orb_extract: image size differs from the handle's planned size");
    return EAO_E_ARG;
  }
  EAO_HIP_CHECK(hipSetDevice(e.dev));
  // the image through pinned staging (one DMA copy), the outputs back in one copy
  EAO_HIP_CHECK(e.stage_in.reserve((size_t)w * hh));
  if (stride == w) {
    e.stage_in.put(gray, (size_t)w * hh);
  } else {
    const size_t o = e.stage_in.put(nullptr, (size_t)w * hh);
    for (int y = 0; y < hh; y++) std::memcpy(e.stage_in.h + o + (size_t)y * w, gray + (size_t)y * stride, w);
  }
  // moved by kernel by default (EAO_ORB_DMA=1: copy-engine transfers): see OrbEngine::image_in
  static const bool dma = [] {
    const char* v = getenv("EAO_ORB_DMA");
    return v && v[0] == '1';
  }();
  if (dma)
    EAO_HIP_CHECK(hipMemcpyAsync(e.d_img, e.stage_in.h, (size_t)w * hh, hipMemcpyHostToDevice, e.stream));
  else if (int rc0 = e.image_in((size_t)w * hh))
    return rc0;
  int rc = e.run(e.d_img, 1, w, e.d_out_kps, e.d_out_desc, e.d_out_cnt, e.cap, e.stream);
  if (rc) return rc;
  EAO_HIP_CHECK(e.stage_out.reserve(e.out_bytes));
  if (dma)
    EAO_HIP_CHECK(hipMemcpyAsync(e.stage_out.h, e.d_out_blk, e.out_bytes, hipMemcpyDeviceToHost, e.stream));
  else if ((rc = e.outputs_out()))
    return rc;
  EAO_HIP_CHECK(hipStreamSynchronize(e.stream));
  const int n = *(const int*)e.stage_out.h;
  *n_out = n;
  if (n > cap) {
    set_error("eao_orb_extract: output capacity too small");
    return EAO_E_CAPACITY;
  }
  if (n > 0) {
    if (kps) std::memcpy(kps, e.stage_out.h + e.out_kps_off, (size_t)n * sizeof(eao_keypoint));
    if (desc) std::memcpy(desc, e.stage_out.h + e.out_desc_off, (size_t)n * 32);
  }
  return EAO_OK;
}

int eao_orb_extract_batch_device(eao_orb* h, const uint8_t* d_frames, int nframes, int pitch,
                                 eao_keypoint* d_kps, uint8_t* d_desc, int32_t* d_counts, int cap,
                                 void* stream) {
  if (!h || !d_frames || !d_kps || !d_desc || !d_counts) return EAO_E_ARG;
  EAO_HIP_CHECK(hipSetDevice(h->e.dev));
  return h->e.run(d_frames, nframes, pitch, (eao_keypoint_dev*)d_kps, d_desc, d_counts, cap,
                  (hipStream_t)stream);
}

int eao_orb_set_timing(eao_orb* h, int on) {
  if (!h) return EAO_E_ARG;
  EAO_HIP_CHECK(hipSetDevice(h->e.dev));
  if (on && !h->e.ev[0])
    for (auto& e : h->e.ev) EAO_HIP_CHECK(hipEventCreate(&e));
  h->e.timing = on != 0;
  return EAO_OK;
}

int eao_orb_stage_ms(eao_orb* h, float* ms, int n) {
  if (!h || !ms || !h->e.timing) return EAO_E_STATE;
  const int k = OrbEngine::kStages;
  EAO_HIP_CHECK(hipEventSynchronize(h->e.ev[k]));
  for (int i = 0; i < k && i < n; i++) EAO_HIP_CHECK(hipEventElapsedTime(&ms[i], h->e.ev[i], h->e.ev[i + 1]));
  return k;
}

int eao_orb_debug_pyramid(eao_orb* h, const uint8_t* gray, uint8_t* out) {
  if (!h || !gray || !out) return EAO_E_ARG;
  OrbEngine& e = h->e;
  EAO_HIP_CHECK(hipSetDevice(e.dev));
  const int w = e.p.width, hh = e.p.height;
  EAO_HIP_CHECK(hipMemcpy(e.d_img, gray, (size_t)w * hh, hipMemcpyHostToDevice));
  // the batch form of the pyramid (k_pyr_tail for the small levels) on this one image; the
  // single-frame extraction's per-level form is checked through its keypoints / descriptors
  const int keep = e.tail_min_frames;
  e.tail_min_frames = 1;
  int rc = e.run(e.d_img, 1, w, e.d_out_kps, e.d_out_desc, e.d_out_cnt, e.cap, e.stream);
  e.tail_min_frames = keep;
  if (rc) return rc;
  EAO_HIP_CHECK(hipStreamSynchronize(e.stream));
  std::memcpy(out, gray, (size_t)w * hh);
  out += (size_t)w * hh;
  for (int l = 1; l < e.p.nlevels; l++) {
    const LevelDev& L = e.levels[l];
    EAO_HIP_CHECK(hipMemcpy2D(out, L.w, e.d_pyr + L.plane_off, L.pitch, L.w, L.h, hipMemcpyDeviceToHost));
    out += (size_t)L.w * L.h;
  }
  return EAO_OK;
}

int eao_color_to_gray_batch_device(const uint8_t* d_color, int nframes, int w, int h, int pitch, int channels,
                                   int rgb, uint8_t* d_gray, int gray_pitch, int device, void* stream) {
  if (!eao_device_ok(device)) {
    set_error("no usable gfx950 device (the engine has no CPU fallback)");
    return EAO_E_NODEVICE;
  }
  EAO_HIP_CHECK(hipSetDevice(device));
  return color_to_gray(d_color, nframes, w, h, pitch, channels, rgb, d_gray, gray_pitch, (hipStream_t)stream);
}

}  // extern "C"
