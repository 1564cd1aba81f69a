// Host cost of a kernel launch on this runtime against the kernel-argument
// size (diagnostic for the C2 host turnaround: the update's first launch
// call took 3.6 us, profiles/r05a_hostgap.json).  Empty kernels, one stream,
// the call timed with CLOCK_MONOTONIC around hipLaunchKernelGGL / hipExtLaunchKernelGGL.
#include <hip/hip_runtime.h>
#include <hip/hip_ext.h>
#include <cstdio>
#include <ctime>
#include <vector>
#include <algorithm>

template <int N> struct Blob { unsigned long long w[N / 8]; };
template <int N> __global__ void k_blob(Blob<N> b, int* out) {
  if (threadIdx.x == 0 && blockIdx.x == 0 && b.w[0] == 12345ull) out[0] = 1;
}
static double now_us() {
  timespec ts; clock_gettime(CLOCK_MONOTONIC, &ts);
  return ts.tv_sec * 1e6 + ts.tv_nsec * 1e-3;
}
template <int N> void run(hipStream_t s, int* out, int grid, bool ext) {
  Blob<N> b{}; b.w[0] = 1;
  std::vector<double> t;
  for (int rep = 0; rep < 400; ++rep) {
    (void)hipStreamSynchronize(s);
    double t0 = now_us();
    if (ext) hipExtLaunchKernelGGL(k_blob<N>, dim3(grid), dim3(256), 0, s, nullptr, nullptr, 0, b, out);
    else hipLaunchKernelGGL(k_blob<N>, dim3(grid), dim3(256), 0, s, b, out);
    double t1 = now_us();
    if (rep >= 50) t.push_back(t1 - t0);
  }
  std::sort(t.begin(), t.end());
  // back-to-back: 4 launches, the time of the 2nd..4th
  std::vector<double> t4;
  for (int rep = 0; rep < 200; ++rep) {
    (void)hipStreamSynchronize(s);
    hipLaunchKernelGGL(k_blob<N>, dim3(grid), dim3(256), 0, s, b, out);
    double t0 = now_us();
    for (int q = 0; q < 3; ++q) hipLaunchKernelGGL(k_blob<N>, dim3(grid), dim3(256), 0, s, b, out);
    double t1 = now_us();
    if (rep >= 20) t4.push_back((t1 - t0) / 3);
  }
  std::sort(t4.begin(), t4.end());
  // launch -> done (stream sync): idle GPU round trip
  std::vector<double> rt;
  for (int rep = 0; rep < 200; ++rep) {
    (void)hipStreamSynchronize(s);
    double t0 = now_us();
    hipLaunchKernelGGL(k_blob<N>, dim3(grid), dim3(256), 0, s, b, out);
    (void)hipStreamSynchronize(s);
    double t1 = now_us();
    if (rep >= 20) rt.push_back(t1 - t0);
  }
  std::sort(rt.begin(), rt.end());
  printf("{\"kernarg_bytes\": %d, \"grid\": %d, \"ext\": %d, \"first_launch_us_p50\": %.2f, \"p10\": %.2f, "
         "\"queued_launch_us_p50\": %.2f, \"launch_to_sync_us_p50\": %.2f}\n",
         N, grid, ext ? 1 : 0, t[t.size() / 2], t[t.size() / 10], t4[t4.size() / 2], rt[rt.size() / 2]);
}
int main() {
  hipStream_t s; hipStreamCreateWithFlags(&s, hipStreamNonBlocking);
  int* out; hipMalloc(&out, 4);
  for (int ext = 0; ext < 2; ++ext) {
    run<16>(s, out, 782, ext);
    run<256>(s, out, 782, ext);
    run<1024>(s, out, 782, ext);
    run<2048>(s, out, 782, ext);
  }
  return 0;
}
