/* Library-internal interface of fk_comm.hip: the RCCL communicator behind
 * the C-ABI's fk_comm (include/findkmer.h), used by the engine's
 * one-collective shard exchange (fk_engine_shard_exchange). */
#pragma once
#include <hip/hip_runtime.h>
#include <stddef.h>
#include <stdint.h>

struct fk_comm;

int fkc_world(const fk_comm *c);
int fkc_rank(const fk_comm *c);
int fkc_device(const fk_comm *c);
/* in-place sum of n int32 over the ranks, enqueued on `s` */
int fkc_allreduce_i32(fk_comm *c, int32_t *buf, size_t n, hipStream_t s);
/* in-place sum of n int32 onto rank `root`, enqueued on `s` */
int fkc_reduce_i32(fk_comm *c, int32_t *buf, size_t n, int root, hipStream_t s);
/* in-place reduce-scatter: the sum of buf[0, world * per_rank) over the
   ranks; rank r receives its block at buf + r * per_rank */
int fkc_reduce_scatter_i32(fk_comm *c, int32_t *buf, size_t per_rank, hipStream_t s);
/* out of place: the sum of send[0, world * per_rank) over the ranks; rank
   r receives its block at buf + r * per_rank (buf's other blocks untouched) */
int fkc_reduce_scatter_from_i32(fk_comm *c, const int32_t *send, int32_t *buf, size_t per_rank, hipStream_t s);
/* all-to-all with per-peer word counts and offsets (ncclSend/ncclRecv in one
   group); fkc_has_alltoallv: this RCCL exports them */
bool fkc_has_alltoallv(const fk_comm *c);
int fkc_alltoallv_i32(fk_comm *c, const int32_t *send, const uint64_t *scount, const uint64_t *sdispl,
                      int32_t *recv, const uint64_t *rcount, const uint64_t *rdispl, hipStream_t s);
