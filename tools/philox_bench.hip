#include <hip/hip_runtime.h>
#include <stdint.h>
__device__ __forceinline__ uint2 ph_a(uint32_t c0, uint32_t c1, uint32_t c2, uint32_t k0, uint32_t k1) {
  uint32_t c3 = 0;
#pragma unroll
  for (int r = 0; r < 10; r++) {
    uint32_t hi0 = __umulhi(0xD2511F53u, c0), lo0 = 0xD2511F53u * c0;
    uint32_t hi1 = __umulhi(0xCD9E8D57u, c2), lo1 = 0xCD9E8D57u * c2;
    uint32_t n0 = hi1 ^ c1 ^ k0, n2 = hi0 ^ c3 ^ k1;
    c0 = n0; c1 = lo1; c2 = n2; c3 = lo0;
    k0 += 0x9E3779B9u; k1 += 0xBB67AE85u;
  }
  return make_uint2(c0, c1);
}
__device__ __forceinline__ uint2 ph_b(uint32_t c0, uint32_t c1, uint32_t c2, uint32_t k0, uint32_t k1) {
  uint32_t c3 = 0;
#pragma unroll
  for (int r = 0; r < 10; r++) {
    const uint64_t p0 = (uint64_t)c0 * 0xD2511F53u, p1 = (uint64_t)c2 * 0xCD9E8D57u;
    uint32_t n0 = (uint32_t)(p1 >> 32) ^ c1 ^ k0, n2 = (uint32_t)(p0 >> 32) ^ c3 ^ k1;
    c0 = n0; c1 = (uint32_t)p1; c2 = n2; c3 = (uint32_t)p0;
    k0 += 0x9E3779B9u; k1 += 0xBB67AE85u;
  }
  return make_uint2(c0, c1);
}
__device__ __forceinline__ uint64_t mad64(uint32_t a, uint32_t b) {
  uint64_t r; uint64_t cc;
  asm("v_mad_u64_u32 %0, %1, %2, %3, 0" : "=v"(r), "=s"(cc) : "v"(a), "v"(b));
  return r;
}
__device__ __forceinline__ uint2 ph_c(uint32_t c0, uint32_t c1, uint32_t c2, uint32_t k0, uint32_t k1) {
  uint32_t c3 = 0;
#pragma unroll
  for (int r = 0; r < 10; r++) {
    const uint64_t p0 = mad64(c0, 0xD2511F53u), p1 = mad64(c2, 0xCD9E8D57u);
    uint32_t n0 = (uint32_t)(p1 >> 32) ^ c1 ^ k0, n2 = (uint32_t)(p0 >> 32) ^ c3 ^ k1;
    c0 = n0; c1 = (uint32_t)p1; c2 = n2; c3 = (uint32_t)p0;
    k0 += 0x9E3779B9u; k1 += 0xBB67AE85u;
  }
  return make_uint2(c0, c1);
}
template <int V>
__global__ void kern(uint2* out, const uint32_t* in, int iters) {
  uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  uint32_t a = in[i], b = i, s = in[i + 1];
  uint2 acc = make_uint2(0, 0);
  for (int it = 0; it < iters; it++) {
    uint2 w = V == 0 ? ph_a(a + it, b, 7, s, s ^ 0x55) : V == 1 ? ph_b(a + it, b, 7, s, s ^ 0x55) : ph_c(a + it, b, 7, s, s ^ 0x55);
    acc.x ^= w.x; acc.y += w.y;
  }
  out[i] = acc;
}
template __global__ void kern<0>(uint2*, const uint32_t*, int);
template __global__ void kern<1>(uint2*, const uint32_t*, int);
template __global__ void kern<2>(uint2*, const uint32_t*, int);
int main() {
  const int N = 1 << 20, IT = 200;
  uint32_t* in; uint2* out[3];
  hipMalloc(&in, (N + 1) * 4);
  for (int v = 0; v < 3; v++) hipMalloc(&out[v], N * 8);
  uint32_t* h = (uint32_t*)malloc((N + 1) * 4);
  for (int i = 0; i <= N; i++) h[i] = i * 2654435761u;
  hipMemcpy(in, h, (N + 1) * 4, hipMemcpyHostToDevice);
  hipEvent_t e0, e1; hipEventCreate(&e0); hipEventCreate(&e1);
  for (int rep = 0; rep < 2; rep++)
  for (int v = 0; v < 3; v++) {
    hipEventRecord(e0);
    if (v == 0) hipLaunchKernelGGL(kern<0>, dim3(N / 256), dim3(256), 0, 0, out[v], in, IT);
    if (v == 1) hipLaunchKernelGGL(kern<1>, dim3(N / 256), dim3(256), 0, 0, out[v], in, IT);
    if (v == 2) hipLaunchKernelGGL(kern<2>, dim3(N / 256), dim3(256), 0, 0, out[v], in, IT);
    hipEventRecord(e1); hipEventSynchronize(e1);
    float ms; hipEventElapsedTime(&ms, e0, e1);
    printf("variant %d: %.3f ms (%.2f Gdraws/s)\n", v, ms, (double)N * IT / ms / 1e6);
  }
  uint2* r[3];
  for (int v = 0; v < 3; v++) { r[v] = (uint2*)malloc(N * 8); hipMemcpy(r[v], out[v], N * 8, hipMemcpyDeviceToHost); }
  int bad = 0;
  for (int i = 0; i < N; i++) bad += r[0][i].x != r[1][i].x || r[0][i].y != r[1][i].y || r[0][i].x != r[2][i].x || r[0][i].y != r[2][i].y;
  printf("mismatches %d\n", bad);
  return 0;
}
