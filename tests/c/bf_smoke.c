/*
 * bf_smoke.c -- a C caller of the libbf ABI (include/bf.h), run by tests/test_c_abi.py on the GPU.
 *
 * Follows the reference's native harness order (common/UnitTest.cpp:28-57: simulate_input -> transfer_HtoD ->
 * run_kernel -> transfer_DtoH -> verify_output; golden checks as BeamformerCoefficientTest.cu:278-420) against
 * tests/golden/c_smoke.bin, which tests/golden/make_c_fixture.py exports from the oracle:
 *   1. bf_reorder                            == the reorder contract, bit for bit
 *   2. bf_coeff_gen                          == the coefficient contract, bit for bit
 *   3. bf_beamform_fused, int8 (Q14)         == the integer contract, bit for bit
 *   4. bf_beamform_fused, f32                within the fp32 tolerance, per element
 *   5. reorder -> coeff_gen -> bf_beamform   == bf_beamform_fused with exact coefficients, bit for bit
 *   6. argument errors come back as BF_ERR_ARG with a message.
 * Prints "bf_smoke OK" and exits 0, or names the first failing check and exits 1.
 *
 *   gcc -std=c11 -O2 -I include tests/c/bf_smoke.c -L dpdk_dc_sand_amd -lbf -Wl,-rpath,$PWD/dpdk_dc_sand_amd
 *   ./build/bf_smoke tests/golden/c_smoke.bin
 */
#include <math.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "bf.h"

#define CHECK(call)                                                                     \
  do {                                                                                  \
    int st_ = (call);                                                                   \
    if (st_ != BF_OK) {                                                                 \
      fprintf(stderr, "%s:%d: %s -> %d: %s\n", __FILE__, __LINE__, #call, st_, bf_last_error()); \
      exit(1);                                                                          \
    }                                                                                   \
  } while (0)

typedef struct {
  int B, A, C, T, M, Ctot, xeng_id, sample_signed;
  double ts, t0, batch_dt;
  float out_scale;
  uint8_t *raw, *reordered;
  float *delays, *coeffs, *beams_f32, *tol_f32;
  int8_t* beams_i8;
  size_t n_raw, n_delays, n_coeffs, n_beams;
} Fixture;

static void read_exact(FILE* f, void* dst, size_t bytes, const char* what) {
  if (fread(dst, 1, bytes, f) != bytes) {
    fprintf(stderr, "fixture truncated reading %s\n", what);
    exit(1);
  }
}

static void* read_array(FILE* f, size_t bytes, const char* what) {
  void* p = malloc(bytes ? bytes : 1);
  if (!p) exit(1);
  read_exact(f, p, bytes, what);
  return p;
}

/* simulate_input(): the reference simulates on the host; here the simulated input is the oracle's fixture. */
static Fixture load_fixture(const char* path) {
  Fixture x;
  FILE* f = fopen(path, "rb");
  if (!f) {
    fprintf(stderr, "cannot open %s\n", path);
    exit(1);
  }
  int32_t hdr[8];
  double dbl[3];
  read_exact(f, hdr, sizeof hdr, "header");
  read_exact(f, dbl, sizeof dbl, "header");
  read_exact(f, &x.out_scale, sizeof x.out_scale, "header");
  x.B = hdr[0], x.A = hdr[1], x.C = hdr[2], x.T = hdr[3], x.M = hdr[4], x.Ctot = hdr[5], x.xeng_id = hdr[6];
  x.sample_signed = hdr[7];
  x.ts = dbl[0], x.t0 = dbl[1], x.batch_dt = dbl[2];
  x.n_raw = (size_t)x.B * x.A * x.C * x.T * 4;
  x.n_delays = (size_t)x.C * x.M * x.A * 4;
  x.n_coeffs = (size_t)x.C * 2 * x.A * 2 * x.M;
  x.n_beams = (size_t)x.B * 2 * x.C * x.T * 2 * x.M;
  x.raw = read_array(f, x.n_raw, "raw");
  x.delays = read_array(f, x.n_delays * 4, "delays");
  x.reordered = read_array(f, x.n_raw, "reordered");
  x.coeffs = read_array(f, x.n_coeffs * 4, "coeffs");
  x.beams_i8 = read_array(f, x.n_beams, "beams_i8");
  x.beams_f32 = read_array(f, x.n_beams * 4, "beams_f32");
  x.tol_f32 = read_array(f, x.n_beams * 4, "tol_f32");
  fclose(f);
  return x;
}

static void* dev_alloc(size_t bytes) {
  void* p = NULL;
  CHECK(bf_malloc(&p, bytes));
  return p;
}

static void fail(const char* what, size_t i) {
  fprintf(stderr, "bf_smoke FAILED: %s (first difference at element %zu)\n", what, i);
  exit(1);
}

int main(int argc, char** argv) {
  if (argc < 2) {
    fprintf(stderr, "usage: %s tests/golden/c_smoke.bin\n", argv[0]);
    return 2;
  }
  Fixture x = load_fixture(argv[1]);
  int ndev = 0;
  CHECK(bf_device_count(&ndev));
  if (ndev < 1) {
    fprintf(stderr, "no GPU\n");
    return 1;
  }
  CHECK(bf_set_device(0));
  void* stream = NULL;
  CHECK(bf_stream_create(&stream));

  /* transfer_HtoD() */
  uint8_t* d_raw = dev_alloc(x.n_raw);
  float* d_delays = dev_alloc(x.n_delays * 4);
  uint8_t* d_reord = dev_alloc(x.n_raw);
  float* d_coeffs = dev_alloc(x.n_coeffs * 4 * 2 * x.B); /* (B, 2, C, 2A, 2M) for the multiply */
  int8_t* d_q = dev_alloc(x.n_beams);
  float* d_y = dev_alloc(x.n_beams * 4);
  float* d_y2 = dev_alloc(x.n_beams * 4);
  CHECK(bf_memcpy_h2d(d_raw, x.raw, x.n_raw, stream));
  CHECK(bf_memcpy_h2d(d_delays, x.delays, x.n_delays * 4, stream));

  /* run_kernel(): the reference chain and the fused operator, with an event around the fused launch */
  void *e0 = NULL, *e1 = NULL;
  CHECK(bf_event_create(&e0));
  CHECK(bf_event_create(&e1));
  CHECK(bf_reorder(d_raw, d_reord, x.B, x.A, x.C, x.T, stream));
  CHECK(bf_coeff_gen(d_delays, d_coeffs, x.B, 2, x.C, x.Ctot, x.A, x.M, x.xeng_id, x.ts, stream));
  CHECK(bf_beamform(d_reord, d_coeffs, d_y2, x.B, 2, x.C, x.T / 16, x.A, x.M, x.sample_signed, stream));
  const int sflag = x.sample_signed ? BF_FUSED_SIGNED : 0;
  CHECK(bf_event_record(e0, stream));
  CHECK(bf_beamform_fused(d_raw, d_delays, 1, d_q, x.B, x.C, x.T, x.A, x.M, x.Ctot, x.xeng_id, x.ts, x.t0,
                          x.batch_dt, sflag | BF_FUSED_OUT_INT8, x.out_scale, stream));
  CHECK(bf_event_record(e1, stream));
  CHECK(bf_beamform_fused(d_raw, d_delays, 1, d_y, x.B, x.C, x.T, x.A, x.M, x.Ctot, x.xeng_id, x.ts, x.t0,
                          x.batch_dt, sflag, 1.0f, stream));

  /* transfer_DtoH() */
  uint8_t* h_reord = malloc(x.n_raw);
  float* h_coeffs = malloc(x.n_coeffs * 4);
  int8_t* h_q = malloc(x.n_beams);
  float* h_y = malloc(x.n_beams * 4);
  float* h_y2 = malloc(x.n_beams * 4);
  CHECK(bf_memcpy_d2h(h_reord, d_reord, x.n_raw, stream));
  CHECK(bf_memcpy_d2h(h_coeffs, d_coeffs, x.n_coeffs * 4, stream)); /* (b, p) = (0, 0) block */
  CHECK(bf_memcpy_d2h(h_q, d_q, x.n_beams, stream));
  CHECK(bf_memcpy_d2h(h_y, d_y, x.n_beams * 4, stream));
  CHECK(bf_stream_synchronize(stream));
  float kernel_ms = 0.0f;
  CHECK(bf_event_elapsed_ms(&kernel_ms, e0, e1));

  /* verify_output() */
  for (size_t i = 0; i < x.n_raw; ++i)
    if (h_reord[i] != x.reordered[i]) fail("bf_reorder != reorder contract", i);
  if (memcmp(h_coeffs, x.coeffs, x.n_coeffs * 4) != 0) {
    for (size_t i = 0; i < x.n_coeffs; ++i)
      if (memcmp(&h_coeffs[i], &x.coeffs[i], 4)) fail("bf_coeff_gen != coefficient contract", i);
  }
  for (size_t i = 0; i < x.n_beams; ++i)
    if (h_q[i] != x.beams_i8[i]) fail("bf_beamform_fused int8 != Q14 integer contract", i);
  for (size_t i = 0; i < x.n_beams; ++i)
    if (!(fabsf(h_y[i] - x.beams_f32[i]) <= x.tol_f32[i])) fail("bf_beamform_fused f32 outside the tolerance", i);

  /* the three-pass chain == the fused operator with exact (float64, reference-order) coefficients */
  CHECK(bf_beamform_fused(d_raw, d_delays, 1, d_y, x.B, x.C, x.T, x.A, x.M, x.Ctot, x.xeng_id, x.ts, 0.0, 0.0,
                          sflag | BF_FUSED_EXACT_COEFF, 1.0f, stream));
  CHECK(bf_memcpy_d2h(h_y, d_y, x.n_beams * 4, stream));
  CHECK(bf_memcpy_d2h(h_y2, d_y2, x.n_beams * 4, stream));
  CHECK(bf_stream_synchronize(stream));
  if (memcmp(h_y, h_y2, x.n_beams * 4) != 0) {
    for (size_t i = 0; i < x.n_beams; ++i)
      if (memcmp(&h_y[i], &h_y2[i], 4)) fail("reorder -> coeff_gen -> beamform != fused exact", i);
  }

  /* errors: a bad shape is BF_ERR_ARG with a message, not an exit */
  if (bf_reorder(d_raw, d_reord, 1, 1, 1, 17, stream) != BF_ERR_ARG || strstr(bf_last_error(), "16") == NULL)
    fail("bf_reorder accepted T = 17", 0);

  CHECK(bf_event_destroy(e0));
  CHECK(bf_event_destroy(e1));
  void* bufs[] = {d_raw, d_delays, d_reord, d_coeffs, d_q, d_y, d_y2};
  for (size_t i = 0; i < sizeof bufs / sizeof bufs[0]; ++i) CHECK(bf_free(bufs[i]));
  CHECK(bf_stream_destroy(stream));
  printf("bf_smoke OK: B=%d A=%d C=%d T=%d M=%d; reorder, coefficients, int8 beams bit-exact; f32 beams within "
         "tolerance; chain == fused exact; fused int8 launch %.3f ms\n",
         x.B, x.A, x.C, x.T, x.M, kernel_ms);
  return 0;
}
