// numa_probe.cpp -- where pinned host memory lands and what that costs the PCIe legs, per NUMA node (round 5).
//
// For every visible GPU: its PCI bus ID and sysfs NUMA node.  Then, for device 0 and every NUMA node n that has CPUs
// this process may run on: bind the thread to node n (numa.h ScopedBind: CPUs + preferred memory node), allocate a
// pinned buffer with hipHostMalloc (default flags, then hipHostMallocNumaUser), report the node of its pages and the
// H2D / D2H rate of 256 MiB copies from it (HIP events, 8 copies after a warm one).  JSON lines on stdout.
//
//   hipcc -O2 -std=c++17 -o tools/numa_probe tools/numa_probe.cpp
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstring>
#include <string>
#include <vector>

#include "../csrc/numa.h"

using namespace kvsep;

#define CK(x)                                                                            \
  do {                                                                                   \
    hipError_t e_ = (x);                                                                 \
    if (e_ != hipSuccess) {                                                              \
      std::fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));                       \
      return 1;                                                                          \
    }                                                                                    \
  } while (0)

static int copy_rate(void* host, void* dev, size_t n, hipStream_t st, double* h2d, double* d2h) {
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  for (int dir = 0; dir < 2; ++dir) {
    auto go = [&] {
      return dir == 0 ? hipMemcpyAsync(dev, host, n, hipMemcpyHostToDevice, st)
                      : hipMemcpyAsync(host, dev, n, hipMemcpyDeviceToHost, st);
    };
    CK(go());
    CK(hipStreamSynchronize(st));
    CK(hipEventRecord(a, st));
    for (int r = 0; r < 8; ++r) CK(go());
    CK(hipEventRecord(b, st));
    CK(hipEventSynchronize(b));
    float ms = 0;
    CK(hipEventElapsedTime(&ms, a, b));
    (dir == 0 ? *h2d : *d2h) = 8.0 * double(n) / (ms * 1e-3) / 1e9;
  }
  (void)hipEventDestroy(a);
  (void)hipEventDestroy(b);
  return 0;
}

int main() {
  int ndev = 0;
  CK(hipGetDeviceCount(&ndev));
  const std::vector<int> allowed = numa::thread_cpus();
  std::printf("{\"devices\": %d, \"allowed_cpus\": \"%s\"}\n", ndev, numa::format_cpulist(allowed).c_str());
  for (int d = 0; d < ndev; ++d) {
    char bus[64] = {};
    CK(hipDeviceGetPCIBusId(bus, sizeof bus, d));
    std::printf("{\"device\": %d, \"pci_bus_id\": \"%s\", \"numa_node\": %d}\n", d, bus, numa::pci_numa_node(bus));
  }
  for (int n = 0; n < 64; ++n) {
    const std::vector<int> nc = numa::node_cpus(n);
    if (nc.empty()) continue;
    std::printf("{\"node\": %d, \"cpulist\": \"%s\", \"allowed\": \"%s\"}\n", n, numa::format_cpulist(nc).c_str(),
                numa::format_cpulist(numa::node_cpus_allowed(n, allowed)).c_str());
  }
  CK(hipSetDevice(0));
  const size_t kBytes = 256ull << 20;
  void* dev = nullptr;
  CK(hipMalloc(&dev, kBytes));
  hipStream_t st;
  CK(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
  for (int n = 0; n < 64; ++n) {
    if (numa::node_cpus_allowed(n, allowed).empty()) continue;
    numa::ScopedBind bind(n);
    for (int numa_user = 0; numa_user < 2; ++numa_user) {
      void* h = nullptr;
      const unsigned flags = numa_user ? hipHostMallocNumaUser : hipHostMallocDefault;
      if (hipHostMalloc(&h, kBytes, flags) != hipSuccess) {
        std::printf("{\"bind_node\": %d, \"numa_user\": %d, \"error\": \"hipHostMalloc failed\"}\n", n, numa_user);
        (void)hipGetLastError();
        continue;
      }
      const int before = numa::page_node(h);
      std::memset(h, 0x5a, kBytes);
      const int first = numa::page_node(h), mid = numa::page_node(static_cast<char*>(h) + kBytes / 2),
                last = numa::page_node(static_cast<char*>(h) + kBytes - 1);
      hipPointerAttribute_t attr{};
      const bool pinned = hipPointerGetAttributes(&attr, h) == hipSuccess && attr.type == hipMemoryTypeHost;
      double h2d = 0, d2h = 0;
      if (copy_rate(h, dev, kBytes, st, &h2d, &d2h)) return 1;
      std::printf("{\"bind_node\": %d, \"bound\": %s, \"numa_user\": %d, \"page_node_untouched\": %d, "
                  "\"page_node\": [%d, %d, %d], \"host_registered\": %s, \"h2d_GBps\": %.1f, \"d2h_GBps\": %.1f}\n",
                  n, bind.bound() ? "true" : "false", numa_user, before, first, mid, last, pinned ? "true" : "false",
                  h2d, d2h);
      std::fflush(stdout);
      CK(hipHostFree(h));
    }
  }
  CK(hipStreamDestroy(st));
  CK(hipFree(dev));
  return 0;
}
