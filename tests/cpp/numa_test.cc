// numa.h and the copier pool's binding on the CPU (tests/test_numa_cpu.py runs it under a faked sysfs topology:
// KVSEP_SYSFS_ROOT with node0 = 0-3, node1 = 4-5,7 and PCI function 0000:aa:00.0 on node 1).
#include <dirent.h>

#include <cstdio>
#include <cstdlib>
#include <fstream>
#include <string>
#include <vector>

#include "copy_pool.h"
#include "numa.h"

using namespace kvsep;

#define CHECK(c)                                                     \
  do {                                                               \
    if (!(c)) {                                                      \
      std::fprintf(stderr, "%s:%d: CHECK(%s)\n", __FILE__, __LINE__, #c); \
      return 1;                                                      \
    }                                                                \
  } while (0)

static std::string task_field(const std::string& tid, const std::string& file, const std::string& key) {
  std::ifstream f("/proc/self/task/" + tid + "/" + file);
  std::string line;
  while (std::getline(f, line)) {
    if (key.empty()) return line;
    if (line.compare(0, key.size(), key) == 0) {
      std::string v = line.substr(key.size());
      while (!v.empty() && (v[0] == ' ' || v[0] == '\t')) v.erase(0, 1);
      return v;
    }
  }
  return "";
}

int main() {
  CHECK((numa::parse_cpulist("0-3,8,10-11") == std::vector<int>{0, 1, 2, 3, 8, 10, 11}));
  CHECK(numa::parse_cpulist("").empty());
  CHECK((numa::parse_cpulist("5") == std::vector<int>{5}));
  CHECK(numa::format_cpulist({0, 1, 2, 3, 8, 10, 11}) == "0-3,8,10-11");
  CHECK(numa::pci_numa_node("0000:AA:00.0") == 1);
  CHECK(numa::pci_numa_node("0000:bb:00.0") == -1);  // sysfs says -1
  CHECK(numa::pci_numa_node("0000:cc:00.0") == -1);  // no such device
  CHECK((numa::node_cpus(1) == std::vector<int>{4, 5, 7}));
  CHECK(numa::node_cpus(9).empty());

  const std::vector<int> before = numa::thread_cpus();
  CHECK((before == std::vector<int>{0, 1, 2, 3, 4, 5, 6, 7}));
  {
    numa::ScopedBind b(1);
    CHECK(b.bound());
    CHECK((numa::thread_cpus() == std::vector<int>{4, 5, 7}));
    // the copier pool of a context placed on node 1: its workers run on node 1's CPUs
    CopyPool pool(3, b.cpus());
    std::vector<uint8_t> src(4 << 20, 7), dst(4 << 20, 0);
    const CopySeg seg{dst.data(), src.data(), src.size()};
    pool.run(&seg, 1);  // 4 units: wakes every worker, so each has bound itself
    CHECK(dst[12345] == 7 && dst.back() == 7);
    int copiers = 0;
    DIR* d = opendir("/proc/self/task");
    CHECK(d);
    while (dirent* e = readdir(d)) {
      if (e->d_name[0] == '.') continue;
      if (task_field(e->d_name, "comm", "") != "kvsep-copy") continue;
      ++copiers;
      const std::string allowed = task_field(e->d_name, "status", "Cpus_allowed_list:");
      if (allowed != "4-5,7") {
        std::fprintf(stderr, "copier %s allowed %s\n", e->d_name, allowed.c_str());
        return 1;
      }
    }
    closedir(d);
    CHECK(copiers == 3);
  }
  CHECK(numa::thread_cpus() == before);  // the scope restores the caller's affinity
  {
    // a cached CPU list (the group's members): bound to that list, intersected with the thread's CPUs,
    // without reading sysfs
    const std::vector<int> cached{5, 6, 42};
    numa::ScopedBind c(1, &cached);
    CHECK(c.bound());
    CHECK((numa::thread_cpus() == std::vector<int>{5, 6}));
  }
  CHECK(numa::thread_cpus() == before);
  {
    numa::ScopedBind none(9);  // unknown node: nothing changes
    CHECK(!none.bound());
    CHECK(numa::thread_cpus() == before);
  }
  {
    numa::set_affinity(0, {0, 1});
    numa::ScopedBind foreign(1);  // node 1 shares no CPU with {0, 1}: nothing changes
    CHECK(!foreign.bound());
    CHECK((numa::thread_cpus() == std::vector<int>{0, 1}));
    numa::set_affinity(0, before);
  }
  std::printf("numa_test ok\n");
  return 0;
}
