/*
 * hiseg_comm.h — the data-parallel gradient exchange of the hiseg training step, on an RCCL communicator that
 * libhiseg owns (hiseg/distributed.py).
 *
 * Replaces, for the collectives issued INSIDE a training step (the bucketed gradient all-reduce and the loss's
 * class-count all-reduce), the torch.distributed calls a reference-side DDP wrapper would make
 * (torch.nn.parallel.DistributedDataParallel over ProcessGroupNCCL; the reference itself trains on one device,
 * train_advanced.py:680-762).  Why not ProcessGroupNCCL: its watchdog thread queries the end event of every
 * collective it tracks, and on ROCm an event query fails with hipErrorCapturedEvent while the stream that event
 * was recorded on is being captured into a HIP graph -- the process group's own communication stream joins every
 * capture that issues a collective, so a whole-step graph capture races the watchdog.  A communicator of our own
 * has no watchdog and no events: the collective is a plain enqueue on the caller's stream, captured like any
 * kernel.  torch.distributed stays the rendezvous (the unique id travels over it) and serves the eager
 * collectives (parameter broadcast, barriers).
 *
 * RCCL is not linked: hiseg_comm_load dlopen()s the librccl the process already uses (torch's), so one RCCL
 * instance serves both torch.distributed and this communicator.
 */
#ifndef HISEG_COMM_H_
#define HISEG_COMM_H_

#include "hiseg.h"

#ifdef __cplusplus
extern "C" {
#endif

typedef void* hiseg_comm_t; /* ncclComm_t */

#define HISEG_COMM_ID_BYTES 128 /* NCCL_UNIQUE_ID_BYTES */

enum hiseg_comm_dtype { HISEG_COMM_F32 = 0, HISEG_COMM_F64 = 1 };
enum hiseg_comm_op { HISEG_COMM_SUM = 0, HISEG_COMM_AVG = 1 };

/* dlopen `path` (NULL: "librccl.so") and resolve the RCCL entry points used below; idempotent. */
int hiseg_comm_load(const char* path);
/* Rank 0: a fresh unique id (HISEG_COMM_ID_BYTES bytes) to hand to every rank. */
int hiseg_comm_unique_id(unsigned char* id_out);
/* Every rank, collectively: a communicator over `nranks` ranks on HIP device `device`. */
int hiseg_comm_init(hiseg_comm_t* comm, int nranks, const unsigned char* id, int rank, int device);
/* In-place all-reduce of `count` elements at `buf` on `stream` (enqueue only; graph-capturable).  AVG divides by
 * the rank count inside the collective. */
int hiseg_comm_all_reduce(hiseg_comm_t comm, void* buf, long long count, int dtype, int op, hiseg_stream_t stream);
int hiseg_comm_destroy(hiseg_comm_t comm);

#ifdef __cplusplus
}
#endif
#endif /* HISEG_COMM_H_ */
