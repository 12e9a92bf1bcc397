// comm.hip -- the multi-GPU exchange of a scoring round:
// RCCL over xGMI, one communicator per context, and the cross-shard top-k
// merge as a HIP kernel.
//
// The reference runs `parallel_factor` independent search instances
// (python/uptune/api.py:400-401) that exchange their results after every
// round (api.sync, python/uptune/api.py:547-553 -> TuningRunManager.sync,
// opentuner/api.py:87-104).  Here the instances are the ranks of one sharded
// round: each scores its own global index range, and two real exchanges exist
//   * an all-gather of every rank's local top-k records, merged identically on
//     every rank (ut_comm_allgather_topk -> k_merge_keep / k_merge_rank);
//   * a broadcast of the per-round history delta from the evaluating rank
//     (ut_comm_bcast_results).
// Payloads are a few KB per round (latency bound): no bucketing, no ring
// tuning; everything is stream-ordered on the context's stream.
//
// Record layout of the all-gather (W 8-byte words per record, record-major):
//   [0] global index (int64, -1 = empty)   [1] score (f64 bits)
//   [2..5] digest (8 big-endian u32 words, two per u64, low word first)
//   [6..6+ncols) the selected configuration's value row (f64 bits; optional)
#include <rccl/rccl.h>
#include <string.h>

#include "ut_internal.h"

namespace ut {

constexpr int MG_NT = 256;   // merge tile: records staged in LDS per pass
constexpr int REC_HDR = 6;   // index, score, 4 digest words

#define UT_RCCL(ctx, call)                                                                      \
  do {                                                                                          \
    ncclResult_t r_ = (call);                                                                   \
    if (r_ != ncclSuccess)                                                                      \
      return ::ut::set_err((ctx), UT_ECOMM, std::string(#call) + ": " + ncclGetErrorString(r_)); \
  } while (0)

__global__ __launch_bounds__(MG_NT) void k_pack_records(int64_t n, const int64_t* __restrict__ idx,
                                                         const double* __restrict__ score,
                                                         const uint32_t* __restrict__ dig,
                                                         const double* __restrict__ rows, int64_t ld_rows,
                                                         int32_t ncols, int32_t W, uint64_t* __restrict__ rec) {
  const int64_t j = (int64_t)blockIdx.x * MG_NT + threadIdx.x;
  if (j >= n) return;
  const int64_t ix = idx ? idx[j] : -1;
  const double s = score ? score[j] : 0.0;
  uint64_t* r = rec + j * W;
  r[0] = (uint64_t)ix;
  r[1] = (uint64_t)__double_as_longlong(s);
  for (int w = 0; w < 4; ++w)
    r[2 + w] = dig ? ((uint64_t)dig[j * 8 + 2 * w] | ((uint64_t)dig[j * 8 + 2 * w + 1] << 32)) : 0ull;
  for (int32_t p = 0; p < ncols; ++p)
    r[REC_HDR + p] = (ix >= 0 && rows) ? (uint64_t)__double_as_longlong(rows[(int64_t)p * ld_rows + j]) : 0ull;
}

__device__ __forceinline__ bool rec_valid(int64_t ix, double s) { return ix >= 0 && s == s; }

// keep[i] = record i is valid and no valid record with the same digest has a
// smaller global index (equal indices: the earlier record).  Threads j < k
// also reset the output slots (empty: idx -1, score -inf, zero digest / row).
__global__ __launch_bounds__(MG_NT) void k_merge_keep(int64_t n, int32_t W, const uint64_t* __restrict__ rec,
                                                       uint8_t* __restrict__ keep, int32_t k,
                                                       int64_t* __restrict__ out_idx, double* __restrict__ out_score,
                                                       uint32_t* __restrict__ out_dig, double* __restrict__ out_rows,
                                                       int64_t ld_out, int32_t ncols) {
  __shared__ int64_t t_ix[MG_NT];
  __shared__ uint64_t t_d[MG_NT][4];
  const int64_t i = (int64_t)blockIdx.x * MG_NT + threadIdx.x;
  if (i < k) {
    if (out_idx) out_idx[i] = -1;
    if (out_score) out_score[i] = -__builtin_inf();
    if (out_dig)
      for (int w = 0; w < 8; ++w) out_dig[i * 8 + w] = 0u;
    if (out_rows)
      for (int32_t p = 0; p < ncols; ++p) out_rows[(int64_t)p * ld_out + i] = 0.0;
  }
  int64_t my = -1;
  uint64_t md[4] = {0, 0, 0, 0};
  if (i < n) {
    const uint64_t* r = rec + i * W;
    my = (int64_t)r[0];
    if (!rec_valid(my, __longlong_as_double((long long)r[1]))) my = -1;
    for (int w = 0; w < 4; ++w) md[w] = r[2 + w];
  }
  bool dup = false;
  for (int64_t base = 0; base < n; base += MG_NT) {
    __syncthreads();
    const int64_t j = base + threadIdx.x;
    if (j < n) {
      const uint64_t* r = rec + j * W;
      const int64_t ix = (int64_t)r[0];
      t_ix[threadIdx.x] = rec_valid(ix, __longlong_as_double((long long)r[1])) ? ix : -1;
      for (int w = 0; w < 4; ++w) t_d[threadIdx.x][w] = r[2 + w];
    } else {
      t_ix[threadIdx.x] = -1;
    }
    __syncthreads();
    if (my >= 0 && !dup) {
      const int lim = (int)((n - base) < MG_NT ? (n - base) : MG_NT);
      for (int t = 0; t < lim; ++t) {
        const int64_t ix = t_ix[t];
        if (ix < 0) continue;
        if (t_d[t][0] != md[0] || t_d[t][1] != md[1] || t_d[t][2] != md[2] || t_d[t][3] != md[3]) continue;
        if (ix < my || (ix == my && base + t < i)) {
          dup = true;
          break;
        }
      }
    }
  }
  if (i < n) keep[i] = (my >= 0 && !dup) ? 1 : 0;
}

// every surviving record's rank among the survivors in (-score, idx) order;
// ranks < k write their record to that output slot
__global__ __launch_bounds__(MG_NT) void k_merge_rank(int64_t n, int32_t W, const uint64_t* __restrict__ rec,
                                                       const uint8_t* __restrict__ keep, int32_t k,
                                                       int64_t* __restrict__ out_idx, double* __restrict__ out_score,
                                                       uint32_t* __restrict__ out_dig, double* __restrict__ out_rows,
                                                       int64_t ld_out, int32_t ncols) {
  __shared__ int64_t t_ix[MG_NT];
  __shared__ double t_s[MG_NT];
  const int64_t i = (int64_t)blockIdx.x * MG_NT + threadIdx.x;
  const bool mine = i < n && keep[i];
  int64_t my = -1;
  double ms = 0.0;
  if (mine) {
    my = (int64_t)rec[i * W];
    ms = __longlong_as_double((long long)rec[i * W + 1]);
  }
  int64_t rank = 0;
  for (int64_t base = 0; base < n; base += MG_NT) {
    __syncthreads();
    const int64_t j = base + threadIdx.x;
    if (j < n && keep[j]) {
      t_ix[threadIdx.x] = (int64_t)rec[j * W];
      t_s[threadIdx.x] = __longlong_as_double((long long)rec[j * W + 1]);
    } else {
      t_ix[threadIdx.x] = -1;
      t_s[threadIdx.x] = 0.0;
    }
    __syncthreads();
    if (mine) {
      const int lim = (int)((n - base) < MG_NT ? (n - base) : MG_NT);
      for (int t = 0; t < lim; ++t) {
        const int64_t ix = t_ix[t];
        if (ix < 0) continue;
        const double s = t_s[t];
        rank += (s > ms || (s == ms && (ix < my || (ix == my && base + t < i)))) ? 1 : 0;
      }
    }
  }
  if (!mine || rank >= k) return;
  const uint64_t* r = rec + i * W;
  if (out_idx) out_idx[rank] = my;
  if (out_score) out_score[rank] = ms;
  if (out_dig)
    for (int w = 0; w < 4; ++w) {
      out_dig[rank * 8 + 2 * w] = (uint32_t)(r[2 + w] & 0xffffffffull);
      out_dig[rank * 8 + 2 * w + 1] = (uint32_t)(r[2 + w] >> 32);
    }
  if (out_rows)
    for (int32_t p = 0; p < ncols; ++p)
      out_rows[(int64_t)p * ld_out + rank] = __longlong_as_double((long long)r[REC_HDR + p]);
}

// broadcast payload of the history delta: [n][5] = value, digest as 4 words
__global__ void k_pack_results(int64_t n, const double* __restrict__ y, const uint32_t* __restrict__ dig,
                               uint64_t* __restrict__ pay) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  pay[i * 5] = (uint64_t)__double_as_longlong(y[i]);
  for (int w = 0; w < 4; ++w)
    pay[i * 5 + 1 + w] = (uint64_t)dig[i * 8 + 2 * w] | ((uint64_t)dig[i * 8 + 2 * w + 1] << 32);
}

__global__ void k_unpack_results(int64_t n, const uint64_t* __restrict__ pay, double* __restrict__ y,
                                 uint32_t* __restrict__ dig) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  if (y) y[i] = __longlong_as_double((long long)pay[i * 5]);
  if (dig)
    for (int w = 0; w < 4; ++w) {
      dig[i * 8 + 2 * w] = (uint32_t)(pay[i * 5 + 1 + w] & 0xffffffffull);
      dig[i * 8 + 2 * w + 1] = (uint32_t)(pay[i * 5 + 1 + w] >> 32);
    }
}

static int merge_records(ut_ctx* c, int64_t n, int32_t W, int32_t k, int32_t ncols, int64_t* out_idx,
                         double* out_score, uint32_t* out_dig, double* out_rows, int64_t ld_out) {
  int rc;
  if ((rc = ensure(c, c->cm_keep, (size_t)(n > 0 ? n : 1)))) return rc;
  const int64_t span = n > k ? n : k;
  hipLaunchKernelGGL(k_merge_keep, dim3(grid1(span, MG_NT)), dim3(MG_NT), 0, c->stream, n, W, c->cm_recv.p,
                     c->cm_keep.p, k, out_idx, out_score, out_dig, out_rows, ld_out, ncols);
  UT_LAUNCH_CHECK(c);
  if (n > 0) {
    hipLaunchKernelGGL(k_merge_rank, dim3(grid1(n, MG_NT)), dim3(MG_NT), 0, c->stream, n, W, c->cm_recv.p,
                       c->cm_keep.p, k, out_idx, out_score, out_dig, out_rows, ld_out, ncols);
    UT_LAUNCH_CHECK(c);
  }
  return 0;
}

static int check_merge_args(ut_ctx* c, int32_t k, int32_t ncols, const double* rows, int64_t ld_rows,
                            int64_t rows_n, double* out_rows, int64_t ld_out) {
  UT_CHECK(c, k >= 1 && k <= (1 << 16), UT_EINVAL, "topk merge: k must be in [1, 65536]");
  UT_CHECK(c, ncols >= 0 && (ncols == 0 || rows), UT_EINVAL, "topk merge: ncols > 0 needs rows");
  UT_CHECK(c, ncols == 0 || ld_rows >= rows_n, UT_EINVAL, "topk merge: ld_rows < the number of records");
  UT_CHECK(c, !out_rows || ncols == 0 || ld_out >= k, UT_EINVAL, "topk merge: ld_out < k");
  return 0;
}

void comm_release(ut_ctx* c) {
  if (c->comm) {
    ncclCommDestroy((ncclComm_t)c->comm);
    c->comm = nullptr;
  }
  c->comm_rank = 0;
  c->comm_size = 1;
  c->cm_agreed_send = c->cm_agreed_recv = 0;
}

}  // namespace ut

using namespace ut;

extern "C" {

int ut_comm_unique_id(uint8_t* id_host) {
  if (!id_host) return UT_EINVAL;
  ncclUniqueId id;
  if (ncclGetUniqueId(&id) != ncclSuccess) return UT_ECOMM;
  static_assert(sizeof(id) == UT_COMM_ID_BYTES, "ncclUniqueId size");
  memcpy(id_host, &id, sizeof(id));
  return 0;
}

int ut_comm_init(ut_ctx* c, int32_t rank, int32_t nranks, const uint8_t* id_host) {
  if (!c) return UT_EINVAL;
  UT_CHECK(c, id_host && nranks >= 1 && rank >= 0 && rank < nranks, UT_EINVAL, "comm_init: bad arguments");
  UT_CHECK(c, c->comm == nullptr, UT_EINVAL, "comm_init: the context already has a communicator");
  UT_HIP(c, hipSetDevice(c->device));
  ncclUniqueId id;
  memcpy(&id, id_host, sizeof(id));
  ncclComm_t comm = nullptr;
  // (the count / agreement words of ut_comm_bcast_results come with the
  // context: nothing is allocated between a rank's entry and the collective init)
  UT_RCCL(c, ncclCommInitRank(&comm, nranks, id, rank));
  c->comm = comm;
  c->comm_rank = rank;
  c->comm_size = nranks;
  return 0;
}

int ut_comm_destroy(ut_ctx* c) {
  if (!c) return UT_EINVAL;
  UT_HIP(c, hipSetDevice(c->device));
  UT_HIP(c, sync_all(c));
  comm_release(c);
  return 0;
}

int ut_comm_info(ut_ctx* c, int32_t* rank, int32_t* nranks) {
  if (!c) return UT_EINVAL;
  if (rank) *rank = c->comm_rank;
  if (nranks) *nranks = c->comm ? c->comm_size : 1;
  return 0;
}

int ut_topk_merge(ut_ctx* c, int64_t n, int32_t k, const int64_t* idx, const double* score, const uint32_t* digest,
                  const double* rows, int64_t ld_rows, int32_t ncols, int64_t* out_idx, double* out_score,
                  uint32_t* out_digest, double* out_rows, int64_t ld_out) {
  if (!c) return UT_EINVAL;
  int rc;
  UT_CHECK(c, n >= 0 && n <= (1 << 20), UT_EINVAL, "topk merge: n must be in [0, 2^20]");
  UT_CHECK(c, n == 0 || (idx && score), UT_EINVAL, "topk merge: NULL idx / score");
  if ((rc = check_merge_args(c, k, ncols, rows, ld_rows, n, out_rows, ld_out))) return rc;
  UT_HIP(c, hipSetDevice(c->device));
  const int32_t W = REC_HDR + ncols;
  if ((rc = ensure(c, c->cm_recv, (size_t)(n > 0 ? n : 1) * W))) return rc;
  if (n > 0) {
    hipLaunchKernelGGL(k_pack_records, dim3(grid1(n, MG_NT)), dim3(MG_NT), 0, c->stream, n, idx, score, digest,
                       rows, ld_rows, ncols, W, c->cm_recv.p);
    UT_LAUNCH_CHECK(c);
  }
  return merge_records(c, n, W, k, ncols, out_idx, out_score, out_digest, out_rows, ld_out);
}

int ut_comm_allgather_topk(ut_ctx* c, int32_t k, const int64_t* idx, const double* score, const uint32_t* digest,
                           const double* rows, int64_t ld_rows, int32_t ncols, int64_t* out_idx, double* out_score,
                           uint32_t* out_digest, double* out_rows, int64_t ld_out) {
  if (!c) return UT_EINVAL;
  int rc;
  UT_CHECK(c, c->comm != nullptr && c->cm_cnt.p != nullptr, UT_EINVAL, "comm_allgather_topk: call ut_comm_init first");
  UT_CHECK(c, idx && score, UT_EINVAL, "comm_allgather_topk: NULL idx / score");
  if ((rc = check_merge_args(c, k, ncols, rows, ld_rows, k, out_rows, ld_out))) return rc;
  UT_HIP(c, hipSetDevice(c->device));
  const int32_t W = REC_HDR + ncols;
  const int64_t n = (int64_t)k * c->comm_size;
  const size_t need_send = (size_t)k * W, need_recv = (size_t)n * W;
  if (need_send > c->cm_agreed_send || need_recv > c->cm_agreed_recv) {
    // the record buffers grow: every rank allocates, then the ranks agree on
    // success (all-reduce MIN of an ok flag) before the all-gather, so a rank
    // that could not allocate makes every rank return UT_ENOMEM instead of
    // leaving its peers inside ncclAllGather (ut_comm_bcast_results' step 2).
    // The agreed capacity is the same on every rank (the same calls in the same
    // order), so every rank takes this branch in the same calls.
    const bool have = ensure(c, c->cm_send, need_send) == 0 && ensure(c, c->cm_recv, need_recv) == 0;
    int64_t ok = have ? 1 : 0;
    UT_HIP(c, hipMemcpyAsync(c->cm_cnt.p + 1, &ok, sizeof(ok), hipMemcpyHostToDevice, c->stream));
    UT_RCCL(c, ncclAllReduce(c->cm_cnt.p + 1, c->cm_cnt.p + 1, 1, ncclInt64, ncclMin, (ncclComm_t)c->comm, c->stream));
    UT_HIP(c, hipMemcpyAsync(&ok, c->cm_cnt.p + 1, sizeof(ok), hipMemcpyDeviceToHost, c->stream));
    UT_HIP(c, hipStreamSynchronize(c->stream));
    if (!ok)
      return set_err(c, UT_ENOMEM, have ? "comm_allgather_topk: another rank could not allocate the records"
                                        : "comm_allgather_topk: no memory for the records");
    c->cm_agreed_send = need_send;
    c->cm_agreed_recv = need_recv;
  }
  hipLaunchKernelGGL(k_pack_records, dim3(grid1(k, MG_NT)), dim3(MG_NT), 0, c->stream, (int64_t)k, idx, score,
                     digest, rows, ld_rows, ncols, W, c->cm_send.p);
  UT_LAUNCH_CHECK(c);
  UT_RCCL(c, ncclAllGather(c->cm_send.p, c->cm_recv.p, (size_t)k * W, ncclUint64, (ncclComm_t)c->comm, c->stream));
  return merge_records(c, n, W, k, ncols, out_idx, out_score, out_digest, out_rows, ld_out);
}

// Every rank takes part in every collective of this call whatever fails
// locally, so no rank is ever left waiting inside one (dist.py's design goal):
//   1. the root broadcasts its count, or -2 when its own arguments are bad
//      (n > cap, missing buffers): every rank then returns UT_EINVAL;
//   2. every rank sizes its payload buffer and the ranks agree on success (an
//      all-reduce MIN of an ok flag): a rank that could not allocate makes
//      all of them return UT_ENOMEM before the payload broadcast;
//   3. the payload broadcast.
int ut_comm_bcast_results(ut_ctx* c, int32_t root, int64_t n, double* y, uint32_t* digest, int64_t cap,
                          int64_t* n_out_host) {
  if (!c) return UT_EINVAL;
  UT_CHECK(c, c->comm != nullptr && c->cm_cnt.p != nullptr, UT_EINVAL, "comm_bcast_results: call ut_comm_init first");
  UT_CHECK(c, root >= 0 && root < c->comm_size, UT_EINVAL, "comm_bcast_results: bad root");
  const bool is_root = c->comm_rank == root;
  const bool root_ok = !is_root || (n >= 0 && cap >= 0 && n <= cap && (n == 0 || (y && digest)));
  UT_HIP(c, hipSetDevice(c->device));
  // 1. the root's count (or the failure sentinel) first
  int64_t cnt = is_root ? (root_ok ? n : -2) : -1;
  UT_HIP(c, hipMemcpyAsync(c->cm_cnt.p, &cnt, sizeof(cnt), hipMemcpyHostToDevice, c->stream));
  UT_RCCL(c, ncclBroadcast(c->cm_cnt.p, c->cm_cnt.p, 1, ncclInt64, root, (ncclComm_t)c->comm, c->stream));
  UT_HIP(c, hipMemcpyAsync(&cnt, c->cm_cnt.p, sizeof(cnt), hipMemcpyDeviceToHost, c->stream));
  UT_HIP(c, hipStreamSynchronize(c->stream));
  if (cnt == -2) {
    if (n_out_host) *n_out_host = 0;
    return set_err(c, UT_EINVAL, is_root ? "comm_bcast_results: the root needs n <= cap and its y / digest buffers"
                                         : "comm_bcast_results: the root's arguments were rejected");
  }
  if (n_out_host) *n_out_host = cnt;
  if (cnt <= 0) return 0;
  // 2. payload buffers on every rank, then agreement
  const bool have = ensure(c, c->cm_pay, (size_t)cnt * 5) == 0;
  int64_t ok = have ? 1 : 0;
  UT_HIP(c, hipMemcpyAsync(c->cm_cnt.p + 1, &ok, sizeof(ok), hipMemcpyHostToDevice, c->stream));
  UT_RCCL(c, ncclAllReduce(c->cm_cnt.p + 1, c->cm_cnt.p + 1, 1, ncclInt64, ncclMin, (ncclComm_t)c->comm, c->stream));
  UT_HIP(c, hipMemcpyAsync(&ok, c->cm_cnt.p + 1, sizeof(ok), hipMemcpyDeviceToHost, c->stream));
  UT_HIP(c, hipStreamSynchronize(c->stream));
  if (!ok)
    return set_err(c, UT_ENOMEM, have ? "comm_bcast_results: another rank could not allocate the payload"
                                      : "comm_bcast_results: no memory for the payload");
  // 3. the payload
  uint64_t* pay = reinterpret_cast<uint64_t*>(c->cm_pay.p);
  if (is_root) {
    hipLaunchKernelGGL(k_pack_results, dim3(grid1(cnt, 256)), dim3(256), 0, c->stream, cnt, y, digest, pay);
    UT_LAUNCH_CHECK(c);
  }
  UT_RCCL(c, ncclBroadcast(pay, pay, (size_t)cnt * 5, ncclUint64, root, (ncclComm_t)c->comm, c->stream));
  const int64_t take = cnt < cap ? cnt : cap;
  if (!is_root && take > 0) {
    hipLaunchKernelGGL(k_unpack_results, dim3(grid1(take, 256)), dim3(256), 0, c->stream, take, pay, y, digest);
    UT_LAUNCH_CHECK(c);
  }
  UT_CHECK(c, cnt <= cap, UT_EINVAL, "comm_bcast_results: the root sent more rows than this rank's capacity");
  return 0;
}

int ut_comm_bcast(ut_ctx* c, void* buf, int64_t bytes, int32_t root) {
  if (!c) return UT_EINVAL;
  UT_CHECK(c, c->comm != nullptr, UT_EINVAL, "comm_bcast: call ut_comm_init first");
  UT_CHECK(c, bytes >= 0 && (buf || bytes == 0) && root >= 0 && root < c->comm_size, UT_EINVAL,
           "comm_bcast: bad arguments");
  if (bytes == 0) return 0;
  UT_HIP(c, hipSetDevice(c->device));
  UT_RCCL(c, ncclBroadcast(buf, buf, (size_t)bytes, ncclUint8, root, (ncclComm_t)c->comm, c->stream));
  return 0;
}

int ut_comm_allreduce_f64(ut_ctx* c, double* buf, int64_t n, int32_t op) {
  if (!c) return UT_EINVAL;
  UT_CHECK(c, c->comm != nullptr, UT_EINVAL, "comm_allreduce: call ut_comm_init first");
  UT_CHECK(c, n >= 0 && (buf || n == 0), UT_EINVAL, "comm_allreduce: bad arguments");
  UT_CHECK(c, op == UT_RED_SUM || op == UT_RED_MAX || op == UT_RED_MIN, UT_EINVAL, "comm_allreduce: bad op");
  if (n == 0) return 0;
  UT_HIP(c, hipSetDevice(c->device));
  const ncclRedOp_t rop = op == UT_RED_SUM ? ncclSum : op == UT_RED_MAX ? ncclMax : ncclMin;
  UT_RCCL(c, ncclAllReduce(buf, buf, (size_t)n, ncclFloat64, rop, (ncclComm_t)c->comm, c->stream));
  return 0;
}

int ut_debug_fail_alloc(ut_ctx* c, int32_t count) {
  if (!c) return UT_EINVAL;
  UT_CHECK(c, count >= 0, UT_EINVAL, "debug_fail_alloc: count < 0");
  c->dbg_fail_alloc = count;
  return 0;
}

int ut_comm_barrier(ut_ctx* c) {
  if (!c) return UT_EINVAL;
  UT_CHECK(c, c->comm != nullptr, UT_EINVAL, "comm_barrier: call ut_comm_init first");
  int rc;
  UT_HIP(c, hipSetDevice(c->device));
  if ((rc = ensure(c, c->cm_cnt, 1))) return rc;
  UT_RCCL(c, ncclAllReduce(c->cm_cnt.p, c->cm_cnt.p, 1, ncclInt64, ncclSum, (ncclComm_t)c->comm, c->stream));
  UT_HIP(c, hipStreamSynchronize(c->stream));
  return 0;
}

}  // extern "C"
