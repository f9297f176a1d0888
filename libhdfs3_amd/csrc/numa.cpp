// NUMA-local placement of each GPU's host-side work (numa.h, docs/DESIGN_HISTORY.md §6).
#include "numa.h"

#include <hip/hip_runtime.h>
#include <pthread.h>

#include <cctype>
#include <cerrno>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <string>

#include "ctx.h"
#include "hdfs3_crc.h"

namespace hdfs3crc {

namespace {

bool read_line(const std::string &path, std::string *out) {
    FILE *f = std::fopen(path.c_str(), "r");
    if (!f) return false;
    char buf[4096];
    const bool ok = std::fgets(buf, sizeof(buf), f) != nullptr;
    std::fclose(f);
    if (!ok) return false;
    *out = buf;
    while (!out->empty() && std::isspace(static_cast<unsigned char>(out->back()))) out->pop_back();
    return true;
}

// "0-31,64-95" -> the set; false on anything else
bool parse_cpulist(const std::string &s, cpu_set_t *out) {
    CPU_ZERO(out);
    size_t i = 0;
    bool any = false;
    while (i < s.size()) {
        char *end = nullptr;
        const long a = std::strtol(s.c_str() + i, &end, 10);
        if (end == s.c_str() + i || a < 0) return false;
        i = size_t(end - s.c_str());
        long b = a;
        if (i < s.size() && s[i] == '-') {
            ++i;
            b = std::strtol(s.c_str() + i, &end, 10);
            if (end == s.c_str() + i || b < a) return false;
            i = size_t(end - s.c_str());
        }
        for (long c = a; c <= b && c < CPU_SETSIZE; ++c) CPU_SET(int(c), out);
        any = true;
        if (i < s.size()) {
            if (s[i] != ',') return false;
            ++i;
        }
    }
    return any;
}

std::string lower(std::string s) {
    for (char &c : s) c = char(std::tolower(static_cast<unsigned char>(c)));
    return s;
}

constexpr int kMaxDevices = 64;
std::once_flag g_once[kMaxDevices];
int g_node[kMaxDevices];
cpu_set_t g_cpus[kMaxDevices];
bool g_have[kMaxDevices];

void lookup(int device) {
    g_node[device] = -1;
    g_have[device] = false;
    char bdf[64] = {0};
    if (hipDeviceGetPCIBusId(bdf, int(sizeof(bdf)), device) != hipSuccess) {
        (void)hipGetLastError();
        return;
    }
    const int node = pci_numa_node("/sys", bdf);
    cpu_set_t want, allowed, both;
    if (node < 0 || !node_cpus("/sys", node, &want)) return;
    if (sched_getaffinity(0, sizeof(allowed), &allowed) != 0) return;
    CPU_AND(&both, &want, &allowed);
    if (CPU_COUNT(&both) == 0) return;  // a cpuset that excludes the node: leave threads alone
    g_node[device] = node;
    g_cpus[device] = both;
    g_have[device] = true;
}

// Opt-in (HDFS3_NUMA=1). Binding the readers' receiver and loader threads to their GPU's node
// measured slower on the one-GPU box, whose loopback datanode and caller threads are not bound:
// 1 GiB through hdfsRead 3.3-7.5 GiB/s with it against 6.4-7.8 without, 8 concurrent hdfsPreads
// 14.7-17.4 against 24.1-34.3 (profiles/r03/reentry/r3e2eab_*). The benefit it is for (host
// data crossing the socket interconnect on 2-socket 8-GPU nodes) is unmeasured here.
bool enabled() {
    static const bool on = [] {
        const char *e = std::getenv("HDFS3_NUMA");
        return e && std::strcmp(e, "1") == 0;
    }();
    return on;
}

}  // namespace

int pci_numa_node(const char *sysfs_root, const char *pci_bdf) {
    if (!sysfs_root || !pci_bdf) return -1;
    std::string v;
    if (!read_line(std::string(sysfs_root) + "/bus/pci/devices/" + lower(pci_bdf) + "/numa_node", &v)) return -1;
    char *end = nullptr;
    const long n = std::strtol(v.c_str(), &end, 10);
    if (end == v.c_str() || *end) return -1;
    return n >= 0 ? int(n) : -1;
}

bool node_cpus(const char *sysfs_root, int node, cpu_set_t *out) {
    if (!sysfs_root || node < 0 || !out) return false;
    std::string v;
    if (!read_line(std::string(sysfs_root) + "/devices/system/node/node" + std::to_string(node) + "/cpulist", &v))
        return false;
    return parse_cpulist(v, out);
}

int bind_thread_to_device(int device) {
    if (!enabled() || device < 0 || device >= kMaxDevices) return -1;
    std::call_once(g_once[device], [device] { lookup(device); });
    if (!g_have[device]) return -1;
    if (pthread_setaffinity_np(pthread_self(), sizeof(cpu_set_t), &g_cpus[device]) != 0) return -1;
    return g_node[device];
}

unsigned pinned_host_flags() { return enabled() ? hipHostMallocNumaUser : hipHostMallocDefault; }

bool numa_binding_enabled() { return enabled(); }

}  // namespace hdfs3crc

extern "C" {

int hdfs3_numa_cpus(const char *sysfs_root, const char *pci_bdf, int *cpus, int max_cpus) {
    if (!sysfs_root || !pci_bdf || (max_cpus > 0 && !cpus) || max_cpus < 0) return hdfs3crc::fail(-EINVAL, "invalid argument");
    const int node = hdfs3crc::pci_numa_node(sysfs_root, pci_bdf);
    if (node < 0) return 0;
    cpu_set_t set;
    if (!hdfs3crc::node_cpus(sysfs_root, node, &set)) return hdfs3crc::fail(-EINVAL, "node %d: no usable cpulist", node);
    int n = 0;
    for (int c = 0; c < CPU_SETSIZE; ++c)
        if (CPU_ISSET(c, &set)) {
            if (n < max_cpus) cpus[n] = c;
            ++n;
        }
    return n;
}

int hdfs3_device_numa_node(int device, int *node) {
    if (!node) return hdfs3crc::fail(-EINVAL, "null node");
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || device < 0 || device >= ndev) {
        (void)hipGetLastError();
        return hdfs3crc::fail(-ENODEV, "device %d not present", device);
    }
    char bdf[64] = {0};
    if (hipDeviceGetPCIBusId(bdf, int(sizeof(bdf)), device) != hipSuccess) {
        (void)hipGetLastError();
        return hdfs3crc::fail(-EIO, "hipDeviceGetPCIBusId(%d) failed", device);
    }
    *node = hdfs3crc::pci_numa_node("/sys", bdf);
    return 0;
}

}  // extern "C"
