// numa.h -- host placement next to a GPU (no HIP; tests build it on the CPU).  A GPU sits on one NUMA node of a
// 2-socket MI355X host (/sys/bus/pci/devices/<bdf>/numa_node); the host legs that feed it -- the thread that stages a
// batch, the copier threads that gather pageable data into the pinned slots, the pinned slots themselves -- belong
// on that node, so the bytes cross no socket link on their way to the GPU's PCIe root.
//
// The topology is read from sysfs under $KVSEP_SYSFS_ROOT (default /sys), so a test can fake it.  Everything here is
// best effort: an unknown node (-1: no sysfs entry, a single-node host) or a node with none of this thread's CPUs
// changes nothing.  Linux only (sched_setaffinity, set_mempolicy/get_mempolicy by syscall: no libnuma needed).
#pragma once
#include <sched.h>
#include <sys/syscall.h>
#include <unistd.h>

#include <cctype>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

namespace kvsep {
namespace numa {

constexpr int kMpolDefault = 0, kMpolPreferred = 1;
constexpr unsigned long kMpolFNode = 1, kMpolFAddr = 2;
constexpr int kMaxNodes = 1024;

inline std::string sysfs_root() {
  const char* r = std::getenv("KVSEP_SYSFS_ROOT");
  return r && *r ? std::string(r) : std::string("/sys");
}

inline bool read_text(const std::string& path, std::string* out) {
  FILE* f = std::fopen(path.c_str(), "r");
  if (!f) return false;
  char buf[4096];
  const size_t n = std::fread(buf, 1, sizeof buf - 1, f);
  std::fclose(f);
  buf[n] = 0;
  *out = buf;
  while (!out->empty() && (out->back() == '\n' || out->back() == ' ')) out->pop_back();
  return true;
}

// "0-3,8,10-11" -> {0,1,2,3,8,10,11}; malformed pieces are skipped.
inline std::vector<int> parse_cpulist(const std::string& s) {
  std::vector<int> out;
  size_t i = 0;
  while (i < s.size()) {
    size_t j = s.find(',', i);
    if (j == std::string::npos) j = s.size();
    const std::string part = s.substr(i, j - i);
    char* e = nullptr;
    const long a = std::strtol(part.c_str(), &e, 10);
    if (e != part.c_str() && a >= 0) {
      long b = a;
      if (*e == '-') b = std::strtol(e + 1, nullptr, 10);
      for (long c = a; c <= b && c < CPU_SETSIZE; ++c) out.push_back(int(c));
    }
    i = j + 1;
  }
  return out;
}

// {0,1,2,3,8,10,11} -> "0-3,8,10-11" (sorted input)
inline std::string format_cpulist(const std::vector<int>& cpus) {
  std::string s;
  for (size_t i = 0; i < cpus.size();) {
    size_t j = i;
    while (j + 1 < cpus.size() && cpus[j + 1] == cpus[j] + 1) ++j;
    if (!s.empty()) s += ',';
    s += std::to_string(cpus[i]);
    if (j > i) s += '-' + std::to_string(cpus[j]);
    i = j + 1;
  }
  return s;
}

// NUMA node of a PCI function ("0000:75:00.0", any case) or -1 when sysfs does not say.
inline int pci_numa_node(const char* bdf) {
  if (!bdf || !*bdf) return -1;
  std::string b(bdf);
  for (char& ch : b) ch = char(std::tolower(static_cast<unsigned char>(ch)));
  std::string t;
  if (!read_text(sysfs_root() + "/bus/pci/devices/" + b + "/numa_node", &t)) return -1;
  char* e = nullptr;
  const long v = std::strtol(t.c_str(), &e, 10);
  return e != t.c_str() && v >= 0 && v < kMaxNodes ? int(v) : -1;
}

inline std::vector<int> node_cpus(int node) {
  std::string t;
  if (node < 0 || !read_text(sysfs_root() + "/devices/system/node/node" + std::to_string(node) + "/cpulist", &t))
    return {};
  return parse_cpulist(t);
}

inline std::vector<int> thread_cpus() {
  cpu_set_t s;
  CPU_ZERO(&s);
  std::vector<int> out;
  if (sched_getaffinity(0, sizeof s, &s) != 0) return out;
  for (int c = 0; c < CPU_SETSIZE; ++c)
    if (CPU_ISSET(c, &s)) out.push_back(c);
  return out;
}

// CPUs of `node` this thread may run on (sorted); empty if none / unknown.
inline std::vector<int> cpus_allowed(const std::vector<int>& nc, const std::vector<int>& allowed) {
  std::vector<int> out;
  for (int c : nc)
    for (int a : allowed)
      if (a == c) {
        out.push_back(c);
        break;
      }
  return out;
}

inline std::vector<int> node_cpus_allowed(int node, const std::vector<int>& allowed) {
  return cpus_allowed(node_cpus(node), allowed);
}

inline bool set_affinity(pid_t tid, const std::vector<int>& cpus) {
  if (cpus.empty()) return false;
  cpu_set_t s;
  CPU_ZERO(&s);
  for (int c : cpus)
    if (c >= 0 && c < CPU_SETSIZE) CPU_SET(c, &s);
  return sched_setaffinity(tid, sizeof s, &s) == 0;
}

// The calling thread's memory policy: -> mode, and the node set in *mask (kMaxNodes bits).
inline int get_policy(unsigned long* mask) {
  int mode = 0;
  if (syscall(SYS_get_mempolicy, &mode, mask, (unsigned long)kMaxNodes, nullptr, 0ul) != 0) return -1;
  return mode;
}

inline bool set_policy(int mode, const unsigned long* mask) {
  return syscall(SYS_set_mempolicy, mode, mode == kMpolDefault ? nullptr : mask,
                 mode == kMpolDefault ? 0ul : (unsigned long)kMaxNodes + 1) == 0;
}

// NUMA node of the page holding p (faulting it in if it was never touched), or -1.
inline int page_node(const void* p) {
  int node = -1;
  if (!p || syscall(SYS_get_mempolicy, &node, nullptr, 0ul, p, kMpolFNode | kMpolFAddr) != 0) return -1;
  return node;
}

// Binds the calling thread to the CPUs of `node` it may run on and makes the node its preferred memory node, for the
// scope; the thread's previous affinity and memory policy come back at scope end.  No-op for node < 0 or a node with
// none of the thread's CPUs.
class ScopedBind {
 public:
  // node_list: the node's CPUs as the caller cached them (null: read from sysfs now)
  explicit ScopedBind(int node, const std::vector<int>* node_list = nullptr) {
    if (node < 0 || node >= kMaxNodes) return;
    prev_cpus_ = thread_cpus();
    cpus_ = node_list ? cpus_allowed(*node_list, prev_cpus_) : node_cpus_allowed(node, prev_cpus_);
    if (cpus_.empty() || !set_affinity(0, cpus_)) {
      cpus_.clear();
      return;
    }
    bound_ = true;
    prev_mode_ = get_policy(prev_mask_);
    unsigned long m[kMaxNodes / (8 * sizeof(unsigned long))] = {};
    m[node / (8 * sizeof(unsigned long))] |= 1ul << (node % (8 * sizeof(unsigned long)));
    policy_set_ = prev_mode_ >= 0 && set_policy(kMpolPreferred, m);
  }
  ~ScopedBind() {
    if (policy_set_) set_policy(prev_mode_, prev_mask_);
    if (bound_) set_affinity(0, prev_cpus_);
  }
  bool bound() const { return bound_; }
  const std::vector<int>& cpus() const { return cpus_; }
  ScopedBind(const ScopedBind&) = delete;
  ScopedBind& operator=(const ScopedBind&) = delete;

 private:
  std::vector<int> prev_cpus_, cpus_;
  unsigned long prev_mask_[kMaxNodes / (8 * sizeof(unsigned long))] = {};
  int prev_mode_ = -1;
  bool bound_ = false, policy_set_ = false;
};

}  // namespace numa
}  // namespace kvsep
