// mlp_phase.hip — per-phase timing of the fused MLP step kernel (csrc/mlp_step.hip)
// built with DOL_MLP_TRACE: thread 0 of every workgroup stamps wall_clock64()
// (100 MHz) at the phase boundaries; prints the mean phase durations and the
// kernel's span.  Config-5 shape by default (1024 agents, 784-128-10, B = 32).
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off -o mlp_phase mlp_phase.hip
#define DOL_MLP_TRACE 1
#include <stdarg.h>
#include <stdio.h>
#include <stdlib.h>
#include <vector>
#include <algorithm>

#include "../distributed-optimization-and-learning_amd/csrc/mlp_step.hip"

namespace dol {
thread_local char g_err[512] = "";
int fail(int code, const char* fmt, ...) {
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(g_err, sizeof(g_err), fmt, ap);
  va_end(ap);
  fprintf(stderr, "%s\n", g_err);
  return code;
}
int check_launch(const char*) { return hipGetLastError() == hipSuccess ? 0 : -1; }
}  // namespace dol

#define CHECK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); exit(1);} } while (0)

int main(int argc, char** argv) {
  const int n = argc > 1 ? atoi(argv[1]) : 1024;
  const int B = 32, d = 784, h = 128, c = 10;
  const int64_t P = int64_t(h) * d + h + c * h + c;
  const int64_t ld = (P + 63) / 64 * 64;
  float *w, *m, *X, *loss, *ws;
  int64_t* y;
  long long* tr;
  CHECK(hipMalloc(&w, n * ld * 4));
  CHECK(hipMalloc(&m, n * ld * 4));
  CHECK(hipMalloc(&X, int64_t(n) * B * d * 4));
  CHECK(hipMalloc(&y, int64_t(n) * B * 8));
  CHECK(hipMalloc(&loss, n * 4));
  CHECK(hipMalloc(&tr, int64_t(n) * 8 * 8));
  CHECK(hipMalloc(&ws, dol_mlp_step_workspace_bytes(n, B, h)));
  std::vector<float> hw(n * ld), hx(int64_t(n) * B * d);
  std::vector<int64_t> hy(int64_t(n) * B);
  srand(1);
  for (auto& v : hw) v = (rand() / float(RAND_MAX) - 0.5f) * 0.1f;
  for (auto& v : hx) v = rand() / float(RAND_MAX) - 0.5f;
  for (auto& v : hy) v = rand() % c;
  CHECK(hipMemcpy(w, hw.data(), hw.size() * 4, hipMemcpyHostToDevice));
  CHECK(hipMemcpy(m, hw.data(), hw.size() * 4, hipMemcpyHostToDevice));
  CHECK(hipMemcpy(X, hx.data(), hx.size() * 4, hipMemcpyHostToDevice));
  CHECK(hipMemcpy(y, hy.data(), hy.size() * 8, hipMemcpyHostToDevice));
  MlpArgs a{w, ld, nullptr, 0, m, ld, nullptr, nullptr, 0, X, int64_t(B) * d, d, y, B, loss,
            B, d, h, c, -0.01f, 0.5f, 0.0f, 2, 1, tr};
  const size_t lds = dol_mlp_step_lds_bytes(B, h, c);
  hipEvent_t e0, e1;
  CHECK(hipEventCreate(&e0));
  CHECK(hipEventCreate(&e1));
  const dim3 g2(unsigned((d + 31) / 32 * ((n + 7) / 8 * 8)));  // the product's dW1 grid (XCD-grouped tiles)
  hipEvent_t e2;
  CHECK(hipEventCreate(&e2));
  if (argc > 2 && argv[2][0] == 'f') {  // the one-kernel step (PH 3): phases F1, F2+CE, B2, B1
    auto k = mlp_fwd_kernel<1, 3, false, false, 5, 3, 25>;
    const size_t lf = sizeof(float) * (fwd_union_floats(B, h, c, 5, true, fused_park_chunks(25, 5)) + h + c + B) + 4 * B;
    CHECK(hipFuncSetAttribute(reinterpret_cast<const void*>(k), hipFuncAttributeMaxDynamicSharedMemorySize, int(lf)));
    for (int it = 0; it < 3; ++it) hipLaunchKernelGGL(k, dim3(n), dim3(kThreads), lf, 0, a, ws);
    CHECK(hipEventRecord(e0));
    hipLaunchKernelGGL(k, dim3(n), dim3(kThreads), lf, 0, a, ws);
    CHECK(hipEventRecord(e1));
    CHECK(hipEventSynchronize(e1));
    float ms;
    CHECK(hipEventElapsedTime(&ms, e0, e1));
    std::vector<long long> ht(int64_t(n) * 8);
    CHECK(hipMemcpy(ht.data(), tr, ht.size() * 8, hipMemcpyDeviceToHost));
    const char* names[] = {"stage+F1", "F2+CE", "B2", "B1+update"};
    double sum[4] = {0, 0, 0, 0};
    for (int i = 0; i < n; ++i)
      for (int p = 0; p < 4; ++p) sum[p] += double(ht[i * 8 + p + 1] - ht[i * 8 + p]);
    printf("fused kernel %.3f ms (%d agents)\n", ms, n);
    for (int p = 0; p < 4; ++p) printf("  %-20s %8.1f us\n", names[p], sum[p] / n / 100.0);
    return 0;
  }
  if (argc > 2 && argv[2][0] == 't') {  // F1 tiles + the per-agent tail (PH 2): phases load, F2+CE, B2
    const size_t lt = sizeof(float) * (fwd_union_floats(B, h, c, 1) + h + c + B) + 4 * B;
    auto k = mlp_fwd_kernel<1, 3, false, false, 1, 2>;
    const dim3 gt(unsigned(h / 32 * ((n + 7) / 8 * 8)));
    for (int it = 0; it < 3; ++it) {
      hipLaunchKernelGGL(mlp_f1_tile_kernel<5>, gt, dim3(64), 0, 0, a, ws, n);
      hipLaunchKernelGGL(k, dim3(n), dim3(kThreads), lt, 0, a, ws);
    }
    hipLaunchKernelGGL(mlp_f1_tile_kernel<5>, gt, dim3(64), 0, 0, a, ws, n);
    CHECK(hipEventRecord(e0));
    hipLaunchKernelGGL(k, dim3(n), dim3(kThreads), lt, 0, a, ws);
    CHECK(hipEventRecord(e1));
    CHECK(hipEventSynchronize(e1));
    float ms;
    CHECK(hipEventElapsedTime(&ms, e0, e1));
    std::vector<long long> ht(int64_t(n) * 8);
    CHECK(hipMemcpy(ht.data(), tr, ht.size() * 8, hipMemcpyDeviceToHost));
    // stamps: 0 start, 1 H + W2 in LDS, 2 after CE, 5 after dW2 (+ its stores issued), 6 after db2 +
    // barrier, 7 after dZ1 + barrier, 3 end (db1, dZ1 -> ws)
    const char* names[] = {"load H, W2", "F2+CE", "B2a dW2", "db2+barrier", "B2b dZ1", "db1+dZ1 out"};
    const int from[] = {0, 1, 2, 5, 6, 7}, to[] = {1, 2, 5, 6, 7, 3};
    double sum[6] = {0, 0, 0, 0, 0, 0};
    long long t0 = ht[0], tend = ht[3];
    for (int i = 0; i < n; ++i) {
      t0 = std::min(t0, ht[i * 8]);
      tend = std::max(tend, ht[i * 8 + 3]);
      for (int p = 0; p < 6; ++p) sum[p] += double(ht[i * 8 + to[p]] - ht[i * 8 + from[p]]);
    }
    printf("tail kernel %.3f ms (%d agents), span(stamps) %.3f ms\n", ms, n, (tend - t0) / 1e5);
    for (int p = 0; p < 6; ++p) printf("  %-20s %8.1f us\n", names[p], sum[p] / n / 100.0);
    int hist[10] = {0};
    for (int i = 0; i < n; ++i) hist[std::min(int(10.0 * (ht[i * 8] - t0) / double(tend - t0 + 1)), 9)]++;
    printf("  WG starts per 10%% of span:");
    for (int b = 0; b < 10; ++b) printf(" %d", hist[b]);
    printf("\n");
    return 0;
  }
  for (int it = 0; it < 3; ++it) {
    hipLaunchKernelGGL((mlp_fwd_kernel<1, 3, false, false>), dim3(n), dim3(kThreads), lds, 0, a, ws);
    hipLaunchKernelGGL((mlp_dw1_kernel<16, 3, false, false, 2, 1>), g2, dim3(kThreads), 0, 0, a, ws, n);
  }
  CHECK(hipEventRecord(e0));
  hipLaunchKernelGGL((mlp_fwd_kernel<1, 3, false, false>), dim3(n), dim3(kThreads), lds, 0, a, ws);
  CHECK(hipEventRecord(e2));
  hipLaunchKernelGGL((mlp_dw1_kernel<16, 3, false, false, 2, 1>), g2, dim3(kThreads), 0, 0, a, ws, n);
  CHECK(hipEventRecord(e1));
  CHECK(hipEventSynchronize(e1));
  float ms, ms_fwd;
  CHECK(hipEventElapsedTime(&ms, e0, e1));
  CHECK(hipEventElapsedTime(&ms_fwd, e0, e2));
  const double bytes_dw1 = double(n) * (4.0 * h * d * 4 + double(B) * d * 4);  // W1, mom in+out, X
  printf("fwd kernel %.3f ms   dw1 kernel %.3f ms (%.0f GB/s on W1+mom in/out + X)\n", ms_fwd, ms - ms_fwd,
         bytes_dw1 / ((ms - ms_fwd) / 1e3) / 1e9);
  std::vector<long long> ht(int64_t(n) * 8);
  CHECK(hipMemcpy(ht.data(), tr, ht.size() * 8, hipMemcpyDeviceToHost));
  const char* names[] = {"stage+F1", "F2+CE", "B2 (dW2,dZ1,db1)"};
  long long t0 = ht[0], tend = ht[3];
  double sum[3] = {0, 0, 0};
  for (int i = 0; i < n; ++i) {
    t0 = std::min(t0, ht[i * 8]);
    tend = std::max(tend, ht[i * 8 + 3]);
    for (int p = 0; p < 3; ++p) sum[p] += double(ht[i * 8 + p + 1] - ht[i * 8 + p]);
  }
  printf("agents %d  both kernels %.3f ms  fwd span(stamps) %.3f ms  mean fwd WG lifetime %.1f us\n", n, ms,
         (tend - t0) / 1e5, (sum[0] + sum[1] + sum[2]) / n / 100.0);
  for (int p = 0; p < 3; ++p) printf("  %-20s %8.1f us\n", names[p], sum[p] / n / 100.0);
  // start-time histogram: how many WGs start within each 10% of the span
  int hist[10] = {0};
  for (int i = 0; i < n; ++i) {
    int b = int(10.0 * (ht[i * 8] - t0) / double(tend - t0 + 1));
    hist[std::min(b, 9)]++;
  }
  printf("  WG starts per 10%% of span:");
  for (int b = 0; b < 10; ++b) printf(" %d", hist[b]);
  printf("\n");
  return 0;
}
