// Internal: NUMA-local placement of the host side of each GPU's work (docs/DESIGN_HISTORY.md §6). On a
// 2-socket 8-GPU node, data that lands in host memory (a datanode socket, RemoteBlockReader.cpp:245;
// a block file, LocalBlockReader.cpp) and goes H2D crosses the socket interconnect for the GPUs of
// the other socket unless the thread that receives it, and the pinned buffer it lands in, sit on the
// GPU's own node. The worker thread of each device (multi_device.cpp), the block readers' receiver
// threads and the local readers' loader threads bind themselves to the CPUs of their device's node
// (intersected with the process's allowed CPUs) before they allocate pinned staging, which then
// follows the thread's node (hipHostMallocNumaUser). Opt-in: only HDFS3_NUMA=1 turns it on. Not installed.
#pragma once

#include <sched.h>

namespace hdfs3crc {

// NUMA node of a PCI function: <root>/bus/pci/devices/<bdf>/numa_node; -1 when absent or unknown
int pci_numa_node(const char *sysfs_root, const char *pci_bdf);
// the CPUs of `node` (<root>/devices/system/node/node<N>/cpulist, e.g. "0-31,64-95"); false when the
// list is missing or malformed
bool node_cpus(const char *sysfs_root, int node, cpu_set_t *out);
// binds the calling thread to the allowed CPUs of `device`'s node (looked up once per device);
// returns the node, or -1 when disabled, unknown or when no allowed CPU is on it (thread unchanged)
int bind_thread_to_device(int device);
// hipHostMalloc flags for pinned staging allocated by a thread bound as above
unsigned pinned_host_flags();
// HDFS3_NUMA=1: binding is on (off by default)
bool numa_binding_enabled();

}  // namespace hdfs3crc
