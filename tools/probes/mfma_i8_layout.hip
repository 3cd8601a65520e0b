// Probe: operand lane maps of v_mfma_i32_16x16x64_i8 (gfx950), with exact integer data.
// A[r][k] = 1 only at (r0, k0); B[k][c] = k + 1000 * c  -> D[r][c] = (r == r0) ? k0 + 1000*c : 0.
// For every lane l and byte j we set the A-fragment byte to 1 for one (l, j) and read which (row, k) it hit.
#include <hip/hip_runtime.h>
#include <cstdio>
typedef int i32x4 __attribute__((ext_vector_type(4)));
typedef int v4i __attribute__((ext_vector_type(4)));

__global__ void probe(int sel_lane, int sel_byte, int* out_rowk) {
  const int lane = threadIdx.x;
  // A fragment: 16 bytes per lane; one-hot at (sel_lane, sel_byte)
  signed char a[16] = {0};
  if (lane == sel_lane) a[sel_byte] = 1;
  // B fragment: lane l supplies B[k][c]; we want B[k][c] = k (for c=0..15) identifying k; use bytes:
  // We don't know the B map either, so make B[k][c] constant 1 for all k,c: then D[r][c] = sum_k A[r][k] = 1 at row r0.
  signed char b[16];
  for (int j = 0; j < 16; ++j) b[j] = 1;
  v4i av, bv;
  __builtin_memcpy(&av, a, 16);
  __builtin_memcpy(&bv, b, 16);
  i32x4 acc = {0, 0, 0, 0};
  acc = __builtin_amdgcn_mfma_i32_16x16x64_i8(av, bv, acc, 0, 0, 0);
  // D layout (dtype-independent, guide): lane l holds D[row (l>>4)*4+i][col l&15]
  for (int i = 0; i < 4; ++i)
    if (acc[i] != 0) atomicAdd(&out_rowk[(lane >> 4) * 4 + i], acc[i]);
}

// Second probe: B map.  A = all ones; B one-hot at (sel_lane, sel_byte): D[r][c] = 1 for column c0 of every row.
__global__ void probeB(int sel_lane, int sel_byte, int* out_col) {
  const int lane = threadIdx.x;
  signed char a[16], b[16] = {0};
  for (int j = 0; j < 16; ++j) a[j] = 1;
  if (lane == sel_lane) b[sel_byte] = 1;
  v4i av, bv;
  __builtin_memcpy(&av, a, 16);
  __builtin_memcpy(&bv, b, 16);
  i32x4 acc = {0, 0, 0, 0};
  acc = __builtin_amdgcn_mfma_i32_16x16x64_i8(av, bv, acc, 0, 0, 0);
  for (int i = 0; i < 4; ++i)
    if (acc[i] != 0 && (lane >> 4) == 0 && i == 0) atomicAdd(&out_col[lane & 15], acc[i]);
}

// Third probe: k pairing. A[r][k] one-hot at (lane la, byte ja); B one-hot at (lane lb, byte jb): D != 0 iff same k.
__global__ void probeK(int la, int ja, int lb, int jb, int* hit) {
  const int lane = threadIdx.x;
  signed char a[16] = {0}, b[16] = {0};
  if (lane == la) a[ja] = 1;
  if (lane == lb) b[jb] = 1;
  v4i av, bv;
  __builtin_memcpy(&av, a, 16);
  __builtin_memcpy(&bv, b, 16);
  i32x4 acc = {0, 0, 0, 0};
  acc = __builtin_amdgcn_mfma_i32_16x16x64_i8(av, bv, acc, 0, 0, 0);
  for (int i = 0; i < 4; ++i)
    if (acc[i] != 0) atomicAdd(hit, 1);
}

int main() {
  int *d;
  hipMalloc(&d, 64 * sizeof(int));
  // A rows: which D row lights up for (lane, byte)
  printf("A map (lane,byte)->row:\n");
  for (int l = 0; l < 64; l += 1) {
    for (int j = 0; j < 16; j += 15) {
      hipMemset(d, 0, 64 * sizeof(int));
      hipLaunchKernelGGL(probe, dim3(1), dim3(64), 0, 0, l, j, d);
      int h[16];
      hipMemcpy(h, d, 16 * sizeof(int), hipMemcpyDeviceToHost);
      int row = -1;
      for (int r = 0; r < 16; ++r) if (h[r]) row = r;
      if (l < 20 || l % 16 == 0) printf(" (%d,%d)->row %d\n", l, j, row);
    }
  }
  printf("B map (lane,byte)->col:\n");
  for (int l = 0; l < 64; l += 5) {
    hipMemset(d, 0, 64 * sizeof(int));
    hipLaunchKernelGGL(probeB, dim3(1), dim3(64), 0, 0, l, 3, d);
    int h[16];
    hipMemcpy(h, d, 16 * sizeof(int), hipMemcpyDeviceToHost);
    int col = -1;
    for (int c = 0; c < 16; ++c) if (h[c]) col = c;
    printf(" (%d,3)->col %d\n", l, col);
  }
  // k pairing: for A lane 0 byte ja, find B (lane lb in {0,16,32,48}, byte jb) giving a hit
  printf("k pairing A(lane0,byte)->B(lane,byte) [A lane l&15=0 row 0; B lane col 0]:\n");
  for (int la = 0; la < 64; la += 16) {
    for (int ja = 0; ja < 16; ++ja) {
      int found_l = -1, found_j = -1;
      for (int lb = 0; lb < 64 && found_l < 0; lb += 16)
        for (int jb = 0; jb < 16; ++jb) {
          hipMemset(d, 0, sizeof(int));
          hipLaunchKernelGGL(probeK, dim3(1), dim3(64), 0, 0, la, ja, lb, jb, d);
          int hit;
          hipMemcpy(&hit, d, sizeof(int), hipMemcpyDeviceToHost);
          if (hit) { found_l = lb; found_j = jb; break; }
        }
      printf(" A(l%d,b%d)~B(l%d,b%d)", la, ja, found_l, found_j);
    }
    printf("\n");
  }
  return 0;
}
