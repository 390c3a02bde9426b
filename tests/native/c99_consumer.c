/* A plain C99 consumer of include/eao_accel.h: the header compiles as C (no C++ types, no
 * extensions: built with -std=c99 -pedantic -Wall -Wextra -Werror) and the library links and runs
 * from C, as a reference-side shim would call it (the reference binds ORBextractor::operator(),
 * include/ORBextractor.h:59-61, and the object association, src/Tracking.cc:1241-1696).
 *
 *   c99_consumer cpu          -- no gfx950 device: every constructor returns EAO_E_NODEVICE
 *   c99_consumer gpu OUT.bin  -- one extraction of a synthetic 640x480 frame (keypoints +
 *                                descriptors written to OUT.bin for the test to compare with the
 *                                oracle), one association replay frame with two boxes
 * Exit status 0 on success; the failing call is printed with eao_last_error(). */
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "eao_accel.h"

#define W 640
#define H 480

static int fail(const char* what, int rc) {
  fprintf(stderr, "%s: rc %d: %s\n", what, rc, eao_last_error());
  return 1;
}

/* the frame the test regenerates in numpy (tests/test_c99_consumer.py: synth_frame) */
static void synth_frame(uint8_t* img) {
  int x, y;
  for (y = 0; y < H; y++)
    for (x = 0; x < W; x++) {
      int v = ((x / 24 + y / 24) & 1) ? 200 : 40;       /* checkerboard: corners at every 24 px */
      v += ((x * 7 + y * 13) & 15) - 8;                  /* texture */
      if ((x - 320) * (x - 320) + (y - 240) * (y - 240) < 90 * 90) v = 255 - v; /* a disc */
      img[y * W + x] = (uint8_t)(v < 0 ? 0 : v > 255 ? 255 : v);
    }
}

static int run_cpu(void) {
  eao_orb_params p;
  eao_orb* orb = NULL;
  eao_assoc* a = NULL;
  int rc;
  memset(&p, 0, sizeof p);
  p.nfeatures = 1000;
  p.scale_factor = 1.2f;
  p.nlevels = 8;
  p.ini_th_fast = 20;
  p.min_th_fast = 7;
  p.width = W;
  p.height = H;
  p.max_batch = 1;
  printf("%s\n", eao_version());
  if (eao_device_ok(0)) return fail("cpu mode: a device is present", 0);
  rc = eao_orb_create(&p, 0, &orb);
  if (rc != EAO_E_NODEVICE || orb) return fail("eao_orb_create without a device", rc);
  rc = eao_assoc_create(0, 4096, &a);
  if (rc != EAO_E_NODEVICE || a) return fail("eao_assoc_create without a device", rc);
  printf("ok: EAO_E_NODEVICE (%s)\n", eao_last_error());
  return 0;
}

static int run_gpu(const char* out_path) {
  eao_orb_params p;
  eao_orb* orb = NULL;
  eao_assoc* a = NULL;
  eao_replay* r = NULL;
  eao_keypoint* kps;
  uint8_t *img, *desc;
  int cap, n = 0, rc, i;
  FILE* f;
  const float K4[4] = {535.4f, 539.2f, 320.1f, 247.6f};
  float Tcw[16];
  int32_t boxes[2 * 5], det[2 * 4];
  int32_t ids[64];
  float pos[64 * 3], uv[64 * 2];
  uint8_t bad[64];
  memset(&p, 0, sizeof p);
  p.nfeatures = 1000;
  p.scale_factor = 1.2f;
  p.nlevels = 8;
  p.ini_th_fast = 20;
  p.min_th_fast = 7;
  p.width = W;
  p.height = H;
  p.max_batch = 1;
  if ((rc = eao_orb_create(&p, 0, &orb)) != EAO_OK) return fail("eao_orb_create", rc);
  cap = eao_orb_frame_capacity(orb);
  img = (uint8_t*)malloc(W * H);
  kps = (eao_keypoint*)malloc(sizeof(eao_keypoint) * (size_t)cap);
  desc = (uint8_t*)malloc(32 * (size_t)cap);
  synth_frame(img);
  if ((rc = eao_orb_extract(orb, img, W, H, W, kps, desc, cap, &n)) != EAO_OK) return fail("eao_orb_extract", rc);
  f = fopen(out_path, "wb");
  if (!f) return fail("open output", 0);
  fwrite(&n, sizeof n, 1, f);
  fwrite(kps, sizeof(eao_keypoint), (size_t)n, f);
  fwrite(desc, 32, (size_t)n, f);
  fclose(f);
  printf("extract: %d keypoints, first (%.2f, %.2f) level %d\n", n, (double)kps[0].x, (double)kps[0].y, kps[0].octave);
  eao_orb_destroy(orb);

  /* one association frame: two boxes {class, x, y, w, h} over 64 map points */
  if ((rc = eao_assoc_create(0, 4096, &a)) != EAO_OK) return fail("eao_assoc_create", rc);
  if ((rc = eao_replay_create(a, "EAO", W, H, K4, &r)) != EAO_OK) return fail("eao_replay_create", rc);
  memset(Tcw, 0, sizeof Tcw);
  Tcw[0] = Tcw[5] = Tcw[10] = Tcw[15] = 1.0f;
  for (i = 0; i < 64; i++) {
    const int b = i & 1;
    ids[i] = i;
    uv[2 * i] = (float)(b ? 400 + (i * 7) % 80 : 100 + (i * 5) % 90);
    uv[2 * i + 1] = (float)(200 + (i * 11) % 70);
    pos[3 * i + 2] = 2.0f + 0.01f * (float)(i % 5);
    pos[3 * i] = (uv[2 * i] - K4[2]) * pos[3 * i + 2] / K4[0];
    pos[3 * i + 1] = (uv[2 * i + 1] - K4[3]) * pos[3 * i + 2] / K4[1];
    bad[i] = 0;
  }
  {
    const int32_t b0[5] = {56, 90, 190, 110, 90}, b1[5] = {62, 390, 190, 100, 90};
    memcpy(boxes, b0, sizeof b0);
    memcpy(boxes + 5, b1, sizeof b1);
  }
  if ((rc = eao_replay_frame(r, 1, Tcw, 2, boxes, 64, ids, pos, uv, bad, det)) < 0) return fail("eao_replay_frame", rc);
  printf("replay: frame 1 -> %d, det %d %d %d %d | %d %d %d %d\n", rc, det[0], det[1], det[2], det[3], det[4], det[5],
         det[6], det[7]);
  eao_replay_destroy(r);
  eao_assoc_destroy(a);
  free(img);
  free(kps);
  free(desc);
  printf("ok\n");
  return 0;
}

int main(int argc, char** argv) {
  if (argc >= 2 && strcmp(argv[1], "cpu") == 0) return run_cpu();
  if (argc >= 3 && strcmp(argv[1], "gpu") == 0) return run_gpu(argv[2]);
  fprintf(stderr, "usage: %s cpu | gpu OUT.bin\n", argv[0]);
  return 2;
}
