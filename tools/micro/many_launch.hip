// many_launch.hip -- does rocprofv3 --pmc survive ~200k dispatches of a small
// kernel?  (The round-4 C5 counter pass died with SIGSEGV inside the HIP launch
// path during the index build's 200k per-list launches: profiles/archive/r04_c5_pmc_crash.log.)
// Same shape as that build: one small kernel launch per "list", each over its own
// slice of one large device buffer.  No library code of yrwi is involved.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>

__global__ void k_touch(const unsigned char* __restrict__ rows, long n, unsigned long* __restrict__ out) {
  const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) out[i] = rows[i * 40] + 1ul;
}

int main(int argc, char** argv) {
  const long lists = argc > 1 ? atol(argv[1]) : 200000;
  const long per = 64;  // postings per list
  unsigned char* rows = nullptr;
  unsigned long* out = nullptr;
  if (hipMalloc(&rows, (size_t)lists * per * 40) != hipSuccess || hipMalloc(&out, (size_t)lists * per * 8) != hipSuccess) {
    fprintf(stderr, "alloc failed\n");
    return 1;
  }
  hipMemset(rows, 1, (size_t)lists * per * 40);
  for (long l = 0; l < lists; l++) {
    hipLaunchKernelGGL(k_touch, dim3(1), dim3(64), 0, 0, rows + (size_t)l * per * 40, per, out + (size_t)l * per);
    if (l % 20000 == 0) {
      hipDeviceSynchronize();
      printf("launched %ld\n", l);
      fflush(stdout);
    }
  }
  hipError_t e = hipDeviceSynchronize();
  printf("done %ld launches: %s\n", lists, hipGetErrorString(e));
  return e == hipSuccess ? 0 : 1;
}
