// Random-gather microbenchmark: bytes moved per gathered element under different
// load cache policies (plain, nontemporal, buffer-load aux bits).  Each variant is
// a separate kernel so rocprofv3 --pmc attributes the L2->HBM request sizes.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <vector>
#include <random>

__global__ void g_plain4(const uint32_t* __restrict__ s, const uint32_t* __restrict__ ix, int n, uint32_t* o) {
  int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) o[i] = s[ix[i]];
}
__global__ void g_nt4(const uint32_t* __restrict__ s, const uint32_t* __restrict__ ix, int n, uint32_t* o) {
  int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) o[i] = __builtin_nontemporal_load(s + ix[i]);
}
template <int AUX>
__global__ void g_buf4(const uint32_t* __restrict__ s, const uint32_t* __restrict__ ix, int n, uint32_t* o, int bytes) {
  int i = blockIdx.x * blockDim.x + threadIdx.x;
  const __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc(const_cast<uint32_t*>(s), 0, bytes, 0x00020000);
  if (i < n) o[i] = __builtin_amdgcn_raw_buffer_load_b32(r, ix[i] * 4, 0, AUX);
}
__global__ void g_plain32(const uint4* __restrict__ s, const uint32_t* __restrict__ ix, int n, uint4* o) {
  int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) {
    const uint4* p = s + 2 * (size_t)ix[i];
    uint4 a = p[0], b = p[1];
    o[i] = make_uint4(a.x ^ b.x, a.y ^ b.y, a.z ^ b.z, a.w ^ b.w);
  }
}
__global__ void g_nt32(const uint4* __restrict__ s, const uint32_t* __restrict__ ix, int n, uint4* o) {
  int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) {
    typedef unsigned int v4u __attribute__((ext_vector_type(4)));
    const v4u* p = reinterpret_cast<const v4u*>(s + 2 * (size_t)ix[i]);
    v4u a = __builtin_nontemporal_load(p), b = __builtin_nontemporal_load(p + 1);
    o[i] = make_uint4(a.x ^ b.x, a.y ^ b.y, a.z ^ b.z, a.w ^ b.w);
  }
}

int main() {
  const size_t words = (size_t)1 << 28;  // 1 GiB of uint32
  const int n = 1 << 24;                 // 16M gathers
  uint32_t *s, *ix, *o;
  hipMalloc(&s, words * 4);
  hipMalloc(&ix, (size_t)n * 4);
  hipMalloc(&o, (size_t)n * 16);
  hipMemset(s, 1, words * 4);
  std::vector<uint32_t> h(n), h32(n);
  std::mt19937_64 g(1);
  for (int i = 0; i < n; i++) h[i] = (uint32_t)(g() % words);
  hipMemcpy(ix, h.data(), (size_t)n * 4, hipMemcpyHostToDevice);
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  auto run = [&](const char* name, auto launch) {
    launch();
    hipDeviceSynchronize();
    hipEventRecord(a);
    for (int r = 0; r < 5; r++) launch();
    hipEventRecord(b);
    hipEventSynchronize(b);
    float ms;
    hipEventElapsedTime(&ms, a, b);
    printf("%-10s %8.1f us/launch  %.2f G gathers/s\n", name, ms * 1000 / 5, n / (ms / 5 * 1e-3) / 1e9);
  };
  dim3 G((n + 255) / 256), B(256);
  run("plain4", [&] { g_plain4<<<G, B>>>(s, ix, n, o); });
  run("nt4", [&] { g_nt4<<<G, B>>>(s, ix, n, o); });
  run("buf4_a0", [&] { g_buf4<0><<<G, B>>>(s, ix, n, o, (int)0x7FFFFFFF); });
  run("buf4_a1", [&] { g_buf4<1><<<G, B>>>(s, ix, n, o, (int)0x7FFFFFFF); });
  run("buf4_a2", [&] { g_buf4<2><<<G, B>>>(s, ix, n, o, (int)0x7FFFFFFF); });
  run("buf4_a3", [&] { g_buf4<3><<<G, B>>>(s, ix, n, o, (int)0x7FFFFFFF); });
  // 32-B records: indices over words/8 records
  for (int i = 0; i < n; i++) h32[i] = h[i] / 8;
  hipMemcpy(ix, h32.data(), (size_t)n * 4, hipMemcpyHostToDevice);
  run("plain32", [&] { g_plain32<<<G, B>>>((const uint4*)s, ix, n, (uint4*)o); });
  run("nt32", [&] { g_nt32<<<G, B>>>((const uint4*)s, ix, n, (uint4*)o); });
  return 0;
}
