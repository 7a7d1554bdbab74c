// Graph shapes for a captured training step with one side-stream branch (the DDP bucket collective):
//   linear    N tiny kernels captured on one stream
//   fork      the same + a one-kernel branch forked on a second stream at N/2 and joined at the end
//             (stream-capture fork/join: one graph, two streams)
//   ext       two LINEAR graphs: the main one records an external event at N/2 and waits on a second
//             external event at the end; the side graph (launched on its own stream after the main one)
//             waits on the first, runs the branch kernel and records the second
//   ext_rec   linear graph + one external event record node only (does an event node alone cost?)
// Prints us per replay.  hipcc --offload-arch=gfx950 -O2 tools/graph_ext_probe.hip -o build/graph_ext_probe
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

#define CK(x)                                                                          \
  do {                                                                                 \
    hipError_t e_ = (x);                                                               \
    if (e_ != hipSuccess) {                                                            \
      std::fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
      std::exit(1);                                                                    \
    }                                                                                  \
  } while (0)

__global__ void bump(float* x) { x[threadIdx.x] += 1.f; }

static float* g_x;
static float* g_y;

static void kernels(hipStream_t s, int n) {
  for (int i = 0; i < n; ++i) bump<<<1, 64, 0, s>>>(g_x);
}

static double time_replays(hipGraphExec_t g, hipGraphExec_t side, hipStream_t s, hipStream_t s2) {
  for (int i = 0; i < 10; ++i) {
    CK(hipGraphLaunch(g, s));
    if (side) CK(hipGraphLaunch(side, s2));
  }
  CK(hipDeviceSynchronize());
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  const int it = 200;
  CK(hipEventRecord(a, s));
  for (int i = 0; i < it; ++i) {
    CK(hipGraphLaunch(g, s));
    if (side) CK(hipGraphLaunch(side, s2));
  }
  CK(hipEventRecord(b, s));
  CK(hipEventSynchronize(b));
  float ms = 0.f;
  CK(hipEventElapsedTime(&ms, a, b));
  CK(hipDeviceSynchronize());
  return 1000.0 * ms / it;
}

int main(int argc, char** argv) {
  const int n = argc > 1 ? std::atoi(argv[1]) : 100;
  CK(hipMalloc(&g_x, 256 * sizeof(float)));
  CK(hipMalloc(&g_y, 256 * sizeof(float)));
  hipStream_t s, s2;
  CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
  CK(hipStreamCreateWithFlags(&s2, hipStreamNonBlocking));
  hipEvent_t fork_ev, join_ev, ready_ev, done_ev;
  CK(hipEventCreateWithFlags(&fork_ev, hipEventDisableTiming));
  CK(hipEventCreateWithFlags(&join_ev, hipEventDisableTiming));
  CK(hipEventCreateWithFlags(&ready_ev, hipEventDisableTiming));
  CK(hipEventCreateWithFlags(&done_ev, hipEventDisableTiming));
  hipGraph_t gr;
  hipGraphExec_t lin, fork, ext_main, ext_side, ext_rec;

  // linear
  CK(hipStreamBeginCapture(s, hipStreamCaptureModeThreadLocal));
  kernels(s, n);
  CK(hipStreamEndCapture(s, &gr));
  CK(hipGraphInstantiate(&lin, gr, nullptr, nullptr, 0));

  // fork / join inside one capture
  CK(hipStreamBeginCapture(s, hipStreamCaptureModeThreadLocal));
  kernels(s, n / 2);
  CK(hipEventRecord(fork_ev, s));
  CK(hipStreamWaitEvent(s2, fork_ev, 0));
  bump<<<1, 64, 0, s2>>>(g_y);
  CK(hipEventRecord(join_ev, s2));
  kernels(s, n - n / 2);
  CK(hipStreamWaitEvent(s, join_ev, 0));
  CK(hipStreamEndCapture(s, &gr));
  CK(hipGraphInstantiate(&fork, gr, nullptr, nullptr, 0));

  // two linear graphs joined by external events
  CK(hipStreamBeginCapture(s, hipStreamCaptureModeThreadLocal));
  kernels(s, n / 2);
  CK(hipEventRecordWithFlags(ready_ev, s, hipEventRecordExternal));
  kernels(s, n - n / 2);
  CK(hipStreamWaitEvent(s, done_ev, hipEventWaitExternal));
  CK(hipStreamEndCapture(s, &gr));
  CK(hipGraphInstantiate(&ext_main, gr, nullptr, nullptr, 0));
  CK(hipStreamBeginCapture(s2, hipStreamCaptureModeThreadLocal));
  CK(hipStreamWaitEvent(s2, ready_ev, hipEventWaitExternal));
  bump<<<1, 64, 0, s2>>>(g_y);
  CK(hipEventRecordWithFlags(done_ev, s2, hipEventRecordExternal));
  CK(hipStreamEndCapture(s2, &gr));
  CK(hipGraphInstantiate(&ext_side, gr, nullptr, nullptr, 0));

  // linear + one external record node
  CK(hipStreamBeginCapture(s, hipStreamCaptureModeThreadLocal));
  kernels(s, n / 2);
  CK(hipEventRecordWithFlags(ready_ev, s, hipEventRecordExternal));
  kernels(s, n - n / 2);
  CK(hipStreamEndCapture(s, &gr));
  CK(hipGraphInstantiate(&ext_rec, gr, nullptr, nullptr, 0));

  const double t_lin = time_replays(lin, nullptr, s, s2);
  const double t_fork = time_replays(fork, nullptr, s, s2);
  const double t_ext = time_replays(ext_main, ext_side, s, s2);
  const double t_rec = time_replays(ext_rec, nullptr, s, s2);
  std::printf("{\"kernels\": %d, \"linear_us\": %.1f, \"fork_us\": %.1f, \"ext_two_graphs_us\": %.1f, "
              "\"linear_plus_ext_record_us\": %.1f}\n",
              n, t_lin, t_fork, t_ext, t_rec);
  return 0;
}
