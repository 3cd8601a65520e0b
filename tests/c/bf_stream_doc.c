/*
 * bf_stream_doc.c -- runs the streaming example of INTEGRATION.md verbatim (the Makefile extracts the block marked
 * `<!-- snippet: stream -->` into build/stream_snippet.inc) on the fixture tests/golden/c_smoke.bin: every frame is
 * the fixture's raw cube, every frame's int8 beams must equal the fixture's (the delay model has zero rates, so the
 * steering time does not change the beams).  Prints "bf_stream_doc OK" and exits 0, else exits 1.
 *
 *   ./build/bf_stream_doc tests/golden/c_smoke.bin [n_frames]
 */
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "bf.h"

static uint8_t* g_raw;
static int8_t* g_expect;
static size_t g_in_bytes, g_out_bytes;
static long long g_consumed, g_bad;

static void fill(void* frame) { memcpy(frame, g_raw, g_in_bytes); }

static void consume(void* beams) {
  ++g_consumed;
  if (memcmp(beams, g_expect, g_out_bytes) != 0) ++g_bad;
}

static void* read_block(FILE* f, size_t bytes) {
  void* p = malloc(bytes);
  if (!p || fread(p, 1, bytes, f) != bytes) {
    fprintf(stderr, "fixture truncated\n");
    exit(1);
  }
  return p;
}

int main(int argc, char** argv) {
  if (argc < 2) {
    fprintf(stderr, "usage: %s tests/golden/c_smoke.bin [n_frames]\n", argv[0]);
    return 2;
  }
  FILE* f = fopen(argv[1], "rb");
  if (!f) return 1;
  int32_t hdr[8];
  double dbl[3];
  float out_scale;
  if (fread(hdr, sizeof hdr, 1, f) != 1 || fread(dbl, sizeof dbl, 1, f) != 1 || fread(&out_scale, 4, 1, f) != 1)
    return 1;
  const int B = hdr[0], A = hdr[1], C = hdr[2], T = hdr[3], M = hdr[4], Ctot = hdr[5], xeng_id = hdr[6];
  const double Ts = dbl[0], t0 = dbl[1], batch_dt = dbl[2];
  const double frame_dt = B * batch_dt;
  g_in_bytes = (size_t)B * A * C * T * 4;
  g_out_bytes = (size_t)B * 2 * C * T * 2 * M;
  g_raw = read_block(f, g_in_bytes);
  float* delays = read_block(f, (size_t)C * M * A * 4 * 4); /* (C, M, A, 4): every channel's model is the same */
  free(read_block(f, g_in_bytes));                          /* reordered */
  free(read_block(f, (size_t)C * 2 * A * 2 * M * 4));       /* coefficients */
  g_expect = read_block(f, g_out_bytes);
  fclose(f);
  const float* host_delays = delays; /* channel 0's (M, A, 4) block = the compact (1, M, A, 4) model */
  const long long n_frames = argc > 2 ? atoll(argv[2]) : 12;

  if (bf_set_device(0) != BF_OK) {
    fprintf(stderr, "no GPU: %s\n", bf_last_error());
    return 1;
  }
  void* frames_in[4];
  void* beams_out[4];
  for (int i = 0; i < 4; ++i) {
    if (bf_host_alloc(&frames_in[i], g_in_bytes) != BF_OK || bf_host_alloc(&beams_out[i], g_out_bytes) != BF_OK) {
      fprintf(stderr, "bf_host_alloc: %s\n", bf_last_error());
      return 1;
    }
  }

#include "stream_snippet.inc"

  for (int i = 0; i < 4; ++i) {
    bf_host_free(frames_in[i]);
    bf_host_free(beams_out[i]);
  }
  if (g_consumed != n_frames || g_bad != 0) {
    fprintf(stderr, "bf_stream_doc FAILED: %lld of %lld frames consumed, %lld differ from the fixture (%s)\n",
            g_consumed, n_frames, g_bad, bf_last_error());
    return 1;
  }
  printf("bf_stream_doc OK: %lld frames (B=%d A=%d C=%d T=%d M=%d) streamed, int8 beams bit-exact\n", n_frames, B, A,
         C, T, M);
  return 0;
}
