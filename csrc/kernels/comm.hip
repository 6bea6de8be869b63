// Native collective engine over RCCL (Horovod core + NCCL -> RCCL over xGMI).
//
// The data-parallel step issues its collectives straight into RCCL on the HIP streams the
// kernels run on, so the whole multi-GPU step (exchanges included) is one capturable sequence
// with no host synchronisation:
//   * all_reduce / all_gather : the flat dense-gradient bucket (Horovod DistributedOptimizer,
//                    HVD:262), grouped with the sparse gradient rows' all-to-all on the step's
//                    main stream (one communicator, host-fixed order);
//   * all_to_all   : fixed-capacity id / row / gradient exchanges of the row-sharded embedding
//                    (every peer block has the same byte size, so no split sizes ever travel
//                    through the host; xGMI is a full mesh, so all 7 peer links run at once).
// The communicator is bootstrapped from a unique id that rank 0 creates and the launcher's
// process group broadcasts (the reference's hvd.init / mpirun rendezvous, HVD:295).
// librccl.so.1 is the RCCL PyTorch already loaded (same SONAME), so one RCCL runs per process.
#include <rccl/rccl.h>
#include <string.h>
#include "common.h"

static int nccl_rc(ncclResult_t r) { return r == ncclSuccess ? 0 : 1000 + (int)r; }

HFM_API int hfm_comm_id_bytes() { return (int)sizeof(ncclUniqueId); }

HFM_API int hfm_comm_unique_id(void* out) {
  ncclUniqueId id;
  const ncclResult_t r = ncclGetUniqueId(&id);
  if (r != ncclSuccess) return nccl_rc(r);
  memcpy(out, &id, sizeof(id));
  return 0;
}

// The calling thread's current HIP device is the communicator's device.
HFM_API int hfm_comm_init(void** comm, int nranks, int rank, const void* id_bytes) {
  ncclUniqueId id;
  memcpy(&id, id_bytes, sizeof(id));
  ncclComm_t c = nullptr;
  const ncclResult_t r = ncclCommInitRank(&c, nranks, id, rank);
  if (r != ncclSuccess) return nccl_rc(r);
  *comm = (void*)c;
  return 0;
}

HFM_API int hfm_comm_destroy(void* comm) {
  if (!comm) return 0;
  return nccl_rc(ncclCommDestroy((ncclComm_t)comm));
}

HFM_API int hfm_comm_allreduce_f32(void* comm, float* buf, size_t n, hipStream_t st) {
  if (n == 0) return 0;
  return nccl_rc(ncclAllReduce(buf, buf, n, ncclFloat32, ncclSum, (ncclComm_t)comm, st));
}

// send/recv: nranks blocks of `bytes_per_peer` bytes each (block p goes to / comes from rank p)
HFM_API int hfm_comm_alltoall(void* comm, const void* send, void* recv, size_t bytes_per_peer,
                              hipStream_t st) {
  if (bytes_per_peer == 0) return 0;
  if (bytes_per_peer % 4 == 0)
    return nccl_rc(ncclAllToAll(send, recv, bytes_per_peer / 4, ncclInt32, (ncclComm_t)comm, st));
  return nccl_rc(ncclAllToAll(send, recv, bytes_per_peer, ncclInt8, (ncclComm_t)comm, st));
}

// The gradient rows' all-to-all and the dense gradients' all-gather of the row-sharded step as ONE
// aggregated RCCL operation (group): the small all-gather shares the all-to-all's launch and
// latency instead of adding its own on the critical path.
HFM_API int hfm_comm_alltoall_allgather(void* comm, const void* send, void* recv, size_t bytes_per_peer,
                                        const void* gsend, void* grecv, size_t gbytes_per_rank,
                                        hipStream_t st) {
  if (bytes_per_peer % 4 || gbytes_per_rank % 4) return (int)hipErrorInvalidValue;
  ncclResult_t r = ncclGroupStart();
  if (r != ncclSuccess) return nccl_rc(r);
  if (bytes_per_peer)
    r = ncclAllToAll(send, recv, bytes_per_peer / 4, ncclInt32, (ncclComm_t)comm, st);
  if (r == ncclSuccess && gbytes_per_rank)
    r = ncclAllGather(gsend, grecv, gbytes_per_rank / 4, ncclInt32, (ncclComm_t)comm, st);
  const ncclResult_t e = ncclGroupEnd();
  return nccl_rc(r != ncclSuccess ? r : e);
}

// recv: nranks blocks of `bytes_per_rank` (block p = rank p's send buffer).  Used for the id
// routing of the NEXT batch on a side stream: captured collectives (all-reduce / all-gather) are
// safe on forked capture streams, where RCCL's peer-to-peer all-to-all is not (ROCm 7 / RCCL 2.26
// segfaults at graph instantiation), so there the routing trades N x bytes for capturability.
HFM_API int hfm_comm_allgather(void* comm, const void* send, void* recv, size_t bytes_per_rank,
                               hipStream_t st) {
  if (bytes_per_rank == 0) return 0;
  if (bytes_per_rank % 4 == 0)
    return nccl_rc(ncclAllGather(send, recv, bytes_per_rank / 4, ncclInt32, (ncclComm_t)comm, st));
  return nccl_rc(ncclAllGather(send, recv, bytes_per_rank, ncclInt8, (ncclComm_t)comm, st));
}

// One step's collectives as ONE aggregated RCCL operation (group), issued on the caller's stream.
// The row-sharded step issues every collective it has through this entry, on its main stream and
// on ONE communicator, at fixed points of the step: the sequence of groups is then the same on
// every rank by construction (no concurrent operations on different communicators, no ordering
// that depends on how graph branches are scheduled onto hardware queues -- the deadlock shape
// RCCL only rules out for a consistent issue order).
// kind 0: all-to-all, `bytes` per peer; 1: all-gather, `bytes` per rank; 2: f32 sum all-reduce
// in place (send == recv allowed), `bytes` in total.
struct CommOp {
  int kind;
  int pad;
  const void* send;
  void* recv;
  size_t bytes;
};

HFM_API int hfm_comm_group(void* comm, const CommOp* ops, int nops, hipStream_t st) {
  for (int i = 0; i < nops; ++i)
    if (ops[i].bytes % 4 || ops[i].kind < 0 || ops[i].kind > 2) return (int)hipErrorInvalidValue;
  ncclResult_t r = ncclGroupStart();
  if (r != ncclSuccess) return nccl_rc(r);
  const ncclComm_t c = (ncclComm_t)comm;
  for (int i = 0; i < nops && r == ncclSuccess; ++i) {
    const CommOp& o = ops[i];
    if (o.bytes == 0) continue;
    if (o.kind == 0)
      r = ncclAllToAll(o.send, o.recv, o.bytes / 4, ncclInt32, c, st);
    else if (o.kind == 1)
      r = ncclAllGather(o.send, o.recv, o.bytes / 4, ncclInt32, c, st);
    else
      r = ncclAllReduce(o.send, o.recv, o.bytes / 4, ncclFloat32, ncclSum, c, st);
  }
  const ncclResult_t e = ncclGroupEnd();
  return nccl_rc(r != ncclSuccess ? r : e);
}

