// Calibration probe for the HBM traffic counters on random record gathers (rasterizer
// over-fetch): what does rocprofv3's FETCH_SIZE report for the rasterizer's access shape -- one 36-byte record
// (float4 + float4 + float at a 64-byte stride) gathered per thread from a table far larger than the caches?
// MI355X_MICROARCH.md: FETCH_SIZE = TCC_EA0_RDREQ x 64 B and reports exactly 1/2 of a wide streaming read (128-B
// requests tallied at 64 B), so bench.py doubles it; whether a gather's requests are tallied the same way decides
// whether the doubled figure over-states the rasterizer's traffic.
//
// Kernels (one launch each, rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE in separate passes):
//   stream_copy : out[i] = in[i] over 256 MB (the streaming reference: FETCH should read 128 MB)
//   gather36    : out[i] = f(rec[idx[i]]) reading 36 B of a 64-B record, 8M random records of a 1 GiB table
//   gather64    : the same, reading all 64 B of the record (4 x float4)
//   gather16    : the same, reading one float4 (16 B) of the record
// Build: hipcc --offload-arch=gfx950 -O3 -o tools/fetch_gather_probe tools/fetch_gather_probe.hip
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <vector>

__global__ void stream_copy(const float4* __restrict__ in, float4* __restrict__ out, long long n) {
  const long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) out[i] = in[i];
}

// gather128: one aligned 128-byte record (a whole L2 line) per thread: one EA request per record if the fabric
// requests are 128 B, two if they are 64 B
__global__ void gather128(const float4* __restrict__ rec, const int* __restrict__ idx, float* __restrict__ out, int n) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const long long g = idx[i] >> 1;
  float s = 0.f;
#pragma unroll
  for (int k = 0; k < 8; ++k) {
    const float4 a = rec[8 * g + k];
    s += a.x + a.y + a.z + a.w;
  }
  out[i] = s;
}

template <int NV>  // 1: 16 B, 3: 36 B (2 float4 + 1 float), 4: 64 B
__global__ void gather(const float4* __restrict__ rec, const int* __restrict__ idx, float* __restrict__ out, int n) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const long long g = idx[i];
  const float4 a = rec[4 * g];
  float s = a.x + a.y + a.z + a.w;
  if (NV >= 3) {
    const float4 b = rec[4 * g + 1];
    s += b.x + b.y + b.z + b.w;
    if (NV == 3) s += reinterpret_cast<const float*>(rec + 4 * g + 2)[0];
  }
  if (NV == 4) {
    const float4 b = rec[4 * g + 1], c = rec[4 * g + 2], d = rec[4 * g + 3];
    s += b.x + b.y + b.z + b.w + c.x + c.y + c.z + c.w + d.x + d.y + d.z + d.w;
  }
  out[i] = s;
}

#define CK(x)                                                                   \
  do {                                                                          \
    hipError_t e_ = (x);                                                        \
    if (e_ != hipSuccess) {                                                     \
      fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));                   \
      return 1;                                                                 \
    }                                                                           \
  } while (0)

int main() {
  const long long nrec = 16ll << 20;  // 16 Mi records x 64 B = 1 GiB
  const int n = 8 << 20;              // 8 Mi gathers
  const long long ncopy = 16ll << 20; // 16 Mi float4 = 256 MB
  float4 *rec, *cin, *cout;
  int* idx;
  float* out;
  CK(hipMalloc(&rec, nrec * 64));
  CK(hipMalloc(&idx, (size_t)n * 4));
  CK(hipMalloc(&out, (size_t)n * 4));
  CK(hipMalloc(&cin, ncopy * 16));
  CK(hipMalloc(&cout, ncopy * 16));
  CK(hipMemset(rec, 0, nrec * 64));
  CK(hipMemset(cin, 0, ncopy * 16));
  std::vector<int> h(n);
  unsigned long long x = 88172645463325252ull;
  for (int i = 0; i < n; ++i) {
    x ^= x << 13; x ^= x >> 7; x ^= x << 17;
    h[i] = (int)(x % (unsigned long long)nrec);
  }
  CK(hipMemcpy(idx, h.data(), (size_t)n * 4, hipMemcpyHostToDevice));
  CK(hipDeviceSynchronize());
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  auto timed = [&](const char* name, auto launch, double bytes) {
    launch();  // warm (TLB)
    hipDeviceSynchronize();
    hipEventRecord(e0);
    launch();
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    float ms = 0.f;
    hipEventElapsedTime(&ms, e0, e1);
    printf("%-12s %8.1f us  algorithmic %8.1f MB  %7.1f GB/s\n", name, ms * 1e3, bytes / 1e6, bytes / ms / 1e6);
  };
  const int tb = 256;
  timed("stream_copy", [&] { stream_copy<<<(unsigned)((ncopy + tb - 1) / tb), tb>>>(cin, cout, ncopy); },
        2.0 * ncopy * 16);
  timed("gather16", [&] { gather<1><<<(n + tb - 1) / tb, tb>>>(rec, idx, out, n); }, n * (4.0 + 16 + 4));
  timed("gather36", [&] { gather<3><<<(n + tb - 1) / tb, tb>>>(rec, idx, out, n); }, n * (4.0 + 36 + 4));
  timed("gather64", [&] { gather<4><<<(n + tb - 1) / tb, tb>>>(rec, idx, out, n); }, n * (4.0 + 64 + 4));
  timed("gather128", [&] { gather128<<<(n + tb - 1) / tb, tb>>>(rec, idx, out, n); }, n * (4.0 + 128 + 4));
  printf("records %lld x 64 B, gathers %d, idx + out %.1f MB\n", nrec, n, n * 8.0 / 1e6);
  return 0;
}
