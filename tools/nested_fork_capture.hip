// Minimal HIP-only reproduction of the nested-fork capture failure
// (VERDICT r01 weak 7): capture on stream m, fork s1 from m, fork s2 from
// s1, join s2 -> s1 -> m, end capture, instantiate, launch. No torch, no
// allocator. Variants: argv[1] = "flat" (m -> s1 only), "nested", "nested_direct"
// (s2 joins m directly), "nested_destroy" (every event destroyed right after
// the wait that consumes it -- what torch's Stream.wait_stream does with its
// temporary event); argv[2] = "global" | "thread" | "relaxed" capture mode;
// argv[3] = "autofree": instantiate with hipGraphInstantiateFlagAutoFreeOnLaunch
// (the flag torch's CUDAGraph::instantiate passes), "priority": the three
// streams made with hipStreamCreateWithPriority (torch's stream pool),
// "memcpy": the s1 and s2 work is a D2D hipMemcpyAsync (torch's copy_),
// "lazyevent": the events are created inside the capture (torch creates an
// Event on its first record).
//   hipcc --offload-arch=gfx950 -O2 tools/nested_fork_capture.hip -o /tmp/nfc && /tmp/nfc nested global
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstring>

#define CK(x)                                                                              \
  do {                                                                                     \
    hipError_t e_ = (x);                                                                   \
    if (e_ != hipSuccess) {                                                                \
      std::printf("{\"step\": \"%s\", \"error\": \"%s\"}\n", #x, hipGetErrorString(e_)); \
      std::fflush(stdout);                                                                 \
      return 1;                                                                            \
    }                                                                                      \
  } while (0)

__global__ void k_add(float* x, float v, int n) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) x[i] += v;
}

static void step(const char* s) {
  std::fprintf(stderr, "step: %s\n", s);
  std::fflush(stderr);
}

int main(int argc, char** argv) {
  const char* variant = argc > 1 ? argv[1] : "nested";
  const char* mode_s = argc > 2 ? argv[2] : "global";
  hipStreamCaptureMode mode = !std::strcmp(mode_s, "thread")    ? hipStreamCaptureModeThreadLocal
                              : !std::strcmp(mode_s, "relaxed") ? hipStreamCaptureModeRelaxed
                                                                : hipStreamCaptureModeGlobal;
  const int n = 1 << 16;
  float *a, *b, *c;
  CK(hipMalloc(&a, n * 4));
  CK(hipMalloc(&b, n * 4));
  CK(hipMalloc(&c, n * 4));
  CK(hipMemset(a, 0, n * 4));
  CK(hipMemset(b, 0, n * 4));
  CK(hipMemset(c, 0, n * 4));
  hipStream_t m, s1, s2;
  const char* opt = argc > 3 ? argv[3] : "";
  if (!std::strcmp(opt, "priority")) {
    CK(hipStreamCreateWithPriority(&m, hipStreamNonBlocking, 0));
    CK(hipStreamCreateWithPriority(&s1, hipStreamNonBlocking, 0));
    CK(hipStreamCreateWithPriority(&s2, hipStreamNonBlocking, 0));
  } else {
    CK(hipStreamCreateWithFlags(&m, hipStreamNonBlocking));
    CK(hipStreamCreateWithFlags(&s1, hipStreamNonBlocking));
    CK(hipStreamCreateWithFlags(&s2, hipStreamNonBlocking));
  }
  hipEvent_t e[6];
  const bool lazy = !std::strcmp(opt, "lazyevent");
  if (!lazy)
    for (auto& x : e) CK(hipEventCreateWithFlags(&x, hipEventDisableTiming));
  const bool mcpy = !std::strcmp(opt, "memcpy");
  const dim3 g(n / 256), blk(256);
  step("begin capture");
  CK(hipStreamBeginCapture(m, mode));
  if (lazy)
    for (auto& x : e) CK(hipEventCreateWithFlags(&x, hipEventDisableTiming));
  hipLaunchKernelGGL(k_add, g, blk, 0, m, a, 1.f, n);
  CK(hipEventRecord(e[0], m));
  CK(hipStreamWaitEvent(s1, e[0], 0));  // fork m -> s1
  if (mcpy) {
    CK(hipMemcpyAsync(b, c, n * 4, hipMemcpyDeviceToDevice, s1));  // b = c (0)
    hipLaunchKernelGGL(k_add, g, blk, 0, s1, b, 2.f, n);
  } else {
    hipLaunchKernelGGL(k_add, g, blk, 0, s1, b, 2.f, n);
  }
  const bool nested = std::strcmp(variant, "flat") != 0;
  const bool destroy = !std::strcmp(variant, "nested_destroy");
  if (destroy) {
    CK(hipEventDestroy(e[0]));
    step("destroyed e0");
  }
  if (nested) {
    CK(hipEventRecord(e[1], s1));
    CK(hipStreamWaitEvent(s2, e[1], 0));  // fork s1 -> s2 (nested)
    if (destroy) CK(hipEventDestroy(e[1]));
    if (mcpy) CK(hipMemcpyAsync(c, b, n * 4, hipMemcpyDeviceToDevice, s2));  // c = b (2)
    hipLaunchKernelGGL(k_add, g, blk, 0, s2, c, 4.f, n);
    CK(hipEventRecord(e[2], s2));
    if (!std::strcmp(variant, "nested_direct")) {
      CK(hipStreamWaitEvent(m, e[2], 0));  // join s2 -> m directly
    } else {
      CK(hipStreamWaitEvent(s1, e[2], 0));  // join s2 -> s1
    }
    if (destroy) CK(hipEventDestroy(e[2]));
  }
  CK(hipEventRecord(e[3], s1));
  CK(hipStreamWaitEvent(m, e[3], 0));  // join s1 -> m
  if (destroy) CK(hipEventDestroy(e[3]));
  hipLaunchKernelGGL(k_add, g, blk, 0, m, a, 8.f, n);
  step("end capture");
  hipGraph_t graph;
  CK(hipStreamEndCapture(m, &graph));
  size_t nodes = 0;
  CK(hipGraphGetNodes(graph, nullptr, &nodes));
  step("instantiate");
  hipGraphExec_t exec;
  if (!std::strcmp(opt, "autofree"))
    CK(hipGraphInstantiateWithFlags(&exec, graph, hipGraphInstantiateFlagAutoFreeOnLaunch));
  else
    CK(hipGraphInstantiate(&exec, graph, nullptr, nullptr, 0));
  step("launch");
  CK(hipGraphLaunch(exec, m));
  CK(hipStreamSynchronize(m));
  float ha = 0, hb = 0, hc = 0;
  CK(hipMemcpy(&ha, a, 4, hipMemcpyDeviceToHost));
  CK(hipMemcpy(&hb, b, 4, hipMemcpyDeviceToHost));
  CK(hipMemcpy(&hc, c, 4, hipMemcpyDeviceToHost));
  std::printf("{\"variant\": \"%s\", \"mode\": \"%s\", \"nodes\": %zu, \"a\": %g, \"b\": %g, \"c\": %g, \"ok\": %s}\n",
              variant, mode_s, nodes, ha, hb, hc,
              (ha == 9.f && hb == 2.f && hc == (nested ? (mcpy ? 6.f : 4.f) : 0.f)) ? "true" : "false");
  CK(hipGraphExecDestroy(exec));
  CK(hipGraphDestroy(graph));
  return 0;
}
