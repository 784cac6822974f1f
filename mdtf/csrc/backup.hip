// Backup workers without a host round trip (SyncReplicasOptimizer replicas_to_aggregate R < N).
//
// Reference: distribute_train.py:146-156 -- TF's SyncReplicasOptimizer applies the first R of N gradient pushes
// of a step and drops the stragglers' as stale.  Here every replica stamps the device's constant 100 MHz clock
// when its backward has finished on the device, the stamps are all-gathered (a tiny collective), and each
// replica ranks itself on the device: contributors are the R earliest (ties by rank).  No host synchronize and
// no store round trip, so the whole step stays capturable in a hipGraph.  The per-replica clock origins are
// calibrated once against the host clock (one node: one host clock), so the stamps compare across GPUs.
#include "mdtf_common.h"

using namespace mdtf;

namespace {

__global__ void stamp_kernel(long long* out) {
  if (threadIdx.x == 0) out[0] = static_cast<long long>(__builtin_amdgcn_s_memrealtime());
}

// mask[0] = 1 if this replica is among the R earliest finishers, else 0; stamps in 10-ns ticks, offsets in ns
__global__ void backup_mask_kernel(const long long* stamps, const long long* offsets, int n, int rank, int R,
                                   float* mask) {
  if (threadIdx.x != 0) return;
  const long long me = stamps[rank] * 10 - offsets[rank];
  int order = 0;
  for (int j = 0; j < n; ++j) {
    const long long t = stamps[j] * 10 - offsets[j];
    if (t < me || (t == me && j < rank)) ++order;
  }
  mask[0] = order < R ? 1.f : 0.f;
}

}  // namespace

MDTF_EXPORT int mdtf_stamp_realtime(long long* out, hipStream_t st) {
  hipLaunchKernelGGL(stamp_kernel, dim3(1), dim3(64), 0, st, out);
  MDTF_LAUNCH_CHECK();
  return 0;
}

MDTF_EXPORT int mdtf_backup_mask(const long long* stamps, const long long* offsets, int n, int rank, int R,
                                 float* mask, hipStream_t st) {
  if (n < 1 || rank < 0 || rank >= n || R < 1) return MDTF_EINVAL;
  hipLaunchKernelGGL(backup_mask_kernel, dim3(1), dim3(64), 0, st, stamps, offsets, n, rank, R, mask);
  MDTF_LAUNCH_CHECK();
  return 0;
}
