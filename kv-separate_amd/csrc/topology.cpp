// topology.cpp -- which GPU a caller runs on and where its host legs belong.
//
// One process per GPU (bench.py, a KVDB rank) or one process over several GPUs (group.cpp) both need the same two
// facts per device: its PCI bus ID, which names the physical GPU (so a multi-GPU run can prove its ranks ran on
// distinct devices), and the NUMA node of its PCI function, next to which its pinned staging, its staging thread and
// its copier threads belong.  The scan this serves is GC / recovery over whole vlogs (db/db_impl.cc:880-951,
// :485-571), whose host round trip crosses the socket link when the staging sits on the far node.
#include <dirent.h>
#include <hip/hip_runtime.h>

#include <cctype>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "../../include/kvsep_crc32c.h"
#include "kvsep_internal.h"
#include "numa.h"

extern "C" {

int kvsep_device_pci_bus_id(int device, char* buf, int len) {
  if (!buf || len < 13) {
    kvsep::set_last_error("pci_bus_id: buffer of at least 13 bytes needed");
    return KVSEP_EINVAL;
  }
  const hipError_t e = hipDeviceGetPCIBusId(buf, len, device);
  if (e != hipSuccess) {
    (void)hipGetLastError();
    kvsep::set_last_error((std::string("hipDeviceGetPCIBusId: ") + hipGetErrorString(e)).c_str());
    return device < 0 ? KVSEP_EINVAL : KVSEP_ENODEV;
  }
  for (char* p = buf; *p; ++p) *p = char(std::tolower(static_cast<unsigned char>(*p)));  // sysfs spelling
  return KVSEP_OK;
}

int kvsep_pci_numa_node(const char* pci_bus_id) { return kvsep::numa::pci_numa_node(pci_bus_id); }

int kvsep_device_numa_node(int device) {
  char bus[64] = {};
  if (kvsep_device_pci_bus_id(device, bus, sizeof bus) != KVSEP_OK) return -1;
  return kvsep::numa::pci_numa_node(bus);
}

int kvsep_numa_node_cpus(int node, int* cpus, int cap) {
  const std::vector<int> c = kvsep::numa::node_cpus(node);
  for (int i = 0; cpus && i < cap && i < int(c.size()); ++i) cpus[i] = c[i];  // (cpus may be null: count only)
  return int(c.size());
}

int kvsep_bind_process_numa(int node) {
  if (node < 0 || node >= kvsep::numa::kMaxNodes) return 0;
  const std::vector<int> cpus = kvsep::numa::node_cpus_allowed(node, kvsep::numa::thread_cpus());
  if (cpus.empty()) return 0;
  // every thread that exists now (the HIP runtime's among them); threads created later inherit from their creator
  int bound = 0;
  if (DIR* d = opendir("/proc/self/task")) {
    while (dirent* e = readdir(d)) {
      if (!std::isdigit(static_cast<unsigned char>(e->d_name[0]))) continue;
      if (kvsep::numa::set_affinity(pid_t(std::atoi(e->d_name)), cpus)) ++bound;
    }
    closedir(d);
  }
  if (!bound && !kvsep::numa::set_affinity(0, cpus)) return 0;
  unsigned long mask[kvsep::numa::kMaxNodes / (8 * sizeof(unsigned long))] = {};
  mask[node / (8 * sizeof(unsigned long))] |= 1ul << (node % (8 * sizeof(unsigned long)));
  kvsep::numa::set_policy(kvsep::numa::kMpolPreferred, mask);  // this thread's later allocations: node first
  return int(cpus.size());
}

int kvsep_host_page_node(const void* p) { return kvsep::numa::page_node(p); }

}  // extern "C"
