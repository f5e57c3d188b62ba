// placement.h -- keep the control plane's host threads on CPUs next to the
// GPU.  A codec flush is a burst of host work on every worker thread; left to
// the scheduler those threads wander over every socket of a large host (and,
// under a CPU quota, get throttled when more of them run than the quota
// allows), so the engine pins the thread that initialises it -- and through
// inheritance every thread created afterwards -- to a slice of the CPUs of
// the device's NUMA node.
#pragma once

#include <vector>

namespace sgpu {

/// Restrict the calling thread to `want` CPUs of the NUMA node of PCI device
/// `pciBusId` ("0000:c1:00.0"), slice `slice` of that node's CPUs (one
/// process per GPU: devices sharing a node take disjoint slices), one CPU per
/// physical core first, never more CPUs than a cgroup CPU quota grants and
/// only CPUs the thread may already use.  SIAMESE_AMD_CPUS overrides: "none"
/// leaves the affinity alone, a list such as "0-7,16" is used as given.
/// Returns the CPUs chosen (empty when the affinity was left unchanged).
std::vector<int> place_near_device(const char* pciBusId, unsigned slice, unsigned want);

} // namespace sgpu
