// Dev micro-benchmark (not product code): memory behaviour of the step kernel's access shapes
// on one MI355X, to calibrate DESIGN.md §6.2's traffic / latency reading.
//
//   memlat chase <bytes_per_lane> <steps> <chains> [lanes]
//       every lane walks <chains> independent dependent-load chains through a private slice
//       of <bytes_per_lane> bytes (random 16-B records), <lanes> (default 131072) lanes in
//       64-lane blocks at two waves per SIMD (the step kernel's shape); prints ns per dependent
//       round trip. With few lanes the memory system is idle: the unloaded latency.
//   memlat scatter16 <records_per_lane>
//       every lane reads <records_per_lane> random 16-B records of an 8 GiB buffer (one
//       128-B line each, no reuse): algorithmic bytes = lanes x records x 16, to compare
//       with rocprofv3 FETCH_SIZE (is the 2x streaming correction right for this shape?).
//   memlat stream16 <MiB>
//       coalesced 16-B-per-lane streaming read of <MiB> (the shape the guide calibrated).
// Build: hipcc --offload-arch=gfx950 -O3 tools/memlat.hip -o build/memlat
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>

#define CHK(e)                                                                         \
  do {                                                                                 \
    hipError_t r_ = (e);                                                               \
    if (r_ != hipSuccess) {                                                            \
      std::fprintf(stderr, "%s: %s\n", #e, hipGetErrorString(r_));                    \
      std::exit(1);                                                                    \
    }                                                                                  \
  } while (0)

static constexpr uint32_t LANES = 131072;

__device__ __forceinline__ uint32_t mix(uint32_t a) {
  a ^= a >> 16; a *= 0x7FEB352Du; a ^= a >> 15; a *= 0x846CA68Bu; a ^= a >> 16;
  return a;
}

// slice of lane l: recs records of 16 B; record r holds the next record index of its chain
__global__ void __launch_bounds__(64, 2) init_chase(uint4* buf, uint32_t recs) {
  const uint64_t l = blockIdx.x * 64ull + threadIdx.x;
  uint4* s = buf + l * recs;
  for (uint32_t r = 0; r < recs; r++) {
    const uint32_t nx = mix(r * 2654435761u + (uint32_t)l) % recs;
    s[r] = make_uint4(nx, r, 0u, 0u);
  }
}

template <int CH>
__global__ void __launch_bounds__(64, 2) chase(const uint4* buf, uint32_t recs, uint32_t steps,
                                                uint32_t* out) {
  extern __shared__ uint32_t lds[];  // only to pin two waves per SIMD, as the step kernel
  const uint64_t l = blockIdx.x * 64ull + threadIdx.x;
  const uint4* s = buf + l * recs;
  uint32_t p[CH];
#pragma unroll
  for (int c = 0; c < CH; c++) p[c] = (uint32_t)(l * 7 + c * 13) % recs;
  for (uint32_t i = 0; i < steps; i++) {
#pragma unroll
    for (int c = 0; c < CH; c++) p[c] = s[p[c]].x;
  }
  uint32_t acc = 0;
#pragma unroll
  for (int c = 0; c < CH; c++) acc += p[c];
  if (acc == 0xFFFFFFFFu) lds[threadIdx.x] = acc;
  out[l] = acc;
}

__global__ void __launch_bounds__(64, 2) scatter16(const uint4* buf, uint64_t lines,
                                                    uint32_t per_lane, uint32_t* out) {
  const uint64_t l = blockIdx.x * 64ull + threadIdx.x;
  uint32_t acc = 0;
  for (uint32_t i = 0; i < per_lane; i += 4) {
    uint4 v[4];
#pragma unroll
    for (int q = 0; q < 4; q++) {
      // a distinct 128-B line per read (no two reads share one): line = hash permutation
      const uint64_t k = (l * per_lane + i + q) * 0x9E3779B97F4A7C15ull;
      const uint64_t line = (k >> 20) % lines;
      v[q] = buf[line * 8 + (k & 7)];
    }
#pragma unroll
    for (int q = 0; q < 4; q++) acc += v[q].x ^ v[q].y ^ v[q].z ^ v[q].w;
  }
  out[l] = acc;
}

__global__ void __launch_bounds__(256) stream16(const uint4* buf, uint64_t n, uint32_t* out) {
  uint32_t acc = 0;
  for (uint64_t i = blockIdx.x * 256ull + threadIdx.x; i < n; i += (uint64_t)gridDim.x * 256ull) {
    const uint4 v = buf[i];
    acc += v.x ^ v.y ^ v.z ^ v.w;
  }
  out[blockIdx.x * 256ull + threadIdx.x] = acc;
}

int main(int argc, char** argv) {
  if (argc < 2) { std::fprintf(stderr, "usage: see header\n"); return 2; }
  const char* mode = argv[1];
  hipEvent_t e0, e1;
  CHK(hipEventCreate(&e0));
  CHK(hipEventCreate(&e1));
  uint32_t* out;
  CHK(hipMalloc(&out, (size_t)LANES * 64 * sizeof(uint32_t)));
  float ms = 0;
  if (!std::strcmp(mode, "chase")) {
    const uint64_t bpl = std::strtoull(argv[2], nullptr, 10);
    const uint32_t steps = (uint32_t)std::atoi(argv[3]), ch = (uint32_t)std::atoi(argv[4]);
    const uint32_t recs = (uint32_t)(bpl / 16);
    const uint32_t lanes = argc > 5 ? (uint32_t)std::atoi(argv[5]) : LANES;
    if (lanes % 64 || lanes > LANES) { std::fprintf(stderr, "lanes: multiple of 64, <= %u\n", LANES); return 2; }
    uint4* buf;
    CHK(hipMalloc(&buf, (size_t)lanes * recs * 16));
    init_chase<<<lanes / 64, 64>>>(buf, recs);
    CHK(hipDeviceSynchronize());
    const size_t lds = 20 * 1024;  // the step kernel's 20 KiB per 64-lane block
    for (int rep = 0; rep < 2; rep++) {
      CHK(hipEventRecord(e0));
      if (ch == 1) chase<1><<<lanes / 64, 64, lds>>>(buf, recs, steps, out);
      else if (ch == 2) chase<2><<<lanes / 64, 64, lds>>>(buf, recs, steps, out);
      else chase<4><<<lanes / 64, 64, lds>>>(buf, recs, steps, out);
      CHK(hipEventRecord(e1));
      CHK(hipEventSynchronize(e1));
      CHK(hipEventElapsedTime(&ms, e0, e1));
    }
    std::printf("chase lanes=%u bytes/lane=%llu footprint=%.2f GB steps=%u chains=%u: %.3f ms, %.1f ns per round "
                "trip, %.1f G loads/s\n",
                lanes, (unsigned long long)bpl, (double)lanes * bpl / 1e9, steps, ch, ms, ms * 1e6 / steps,
                (double)lanes * steps * ch / (ms * 1e6));
    CHK(hipFree(buf));
  } else if (!std::strcmp(mode, "scatter16")) {
    const uint32_t per = (uint32_t)std::atoi(argv[2]);
    const uint64_t bytes = 8ull << 30, lines = bytes / 128;
    uint4* buf;
    CHK(hipMalloc(&buf, bytes));
    CHK(hipMemset(buf, 1, bytes));
    CHK(hipDeviceSynchronize());
    CHK(hipEventRecord(e0));
    scatter16<<<LANES / 64, 64>>>(buf, lines, per, out);
    CHK(hipEventRecord(e1));
    CHK(hipEventSynchronize(e1));
    CHK(hipEventElapsedTime(&ms, e0, e1));
    const double alg = (double)LANES * per * 16;
    std::printf("scatter16 records/lane=%u: algorithmic read bytes %.6e, %.3f ms, %.1f GB/s algorithmic\n",
                per, alg, ms, alg / (ms * 1e6));
    CHK(hipFree(buf));
  } else if (!std::strcmp(mode, "stream16")) {
    const uint64_t bytes = std::strtoull(argv[2], nullptr, 10) << 20, n = bytes / 16;
    uint4* buf;
    CHK(hipMalloc(&buf, bytes));
    CHK(hipMemset(buf, 1, bytes));
    CHK(hipDeviceSynchronize());
    CHK(hipEventRecord(e0));
    stream16<<<LANES * 64 / 256, 256>>>(buf, n, out);
    CHK(hipEventRecord(e1));
    CHK(hipEventSynchronize(e1));
    CHK(hipEventElapsedTime(&ms, e0, e1));
    std::printf("stream16: algorithmic read bytes %.6e, %.3f ms, %.1f GB/s\n", (double)bytes, ms,
                bytes / (ms * 1e6));
    CHK(hipFree(buf));
  }
  CHK(hipFree(out));
  return 0;
}
