// insitu.cpp -- the in-situ (domain-sharded) tracer of one rank, with its
// exchange, on the engine's stream: the device form of
// insitu::MultiThreadTracer::traceInOmp (src/insitu/
// insitu_multithread_tracer.inl:313-442) with the MPI queues of Comm::run
// (insitu_comm.inl:28-101) and WorkStats::reduce (insitu_work_stats.cc:34-85)
// replaced by count-first all-to-all-v exchanges over RCCL (or host
// callbacks, spray_rt_transport).  See include/spray_rt.h for the protocol.
//
// Differences from the reference that do not change results: the owners
// learn the composite minimum of each ray copy before shading (the
// reference shades every local hit speculatively and discards the losers
// at VBuf::compositeTbuf), and a fixed number of bounces replaces the
// WorkStats termination test (no rays exist past shader->bounces).
#include <dlfcn.h>
#include <fcntl.h>
#include <sys/file.h>
#include <unistd.h>
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <algorithm>
#include <cstddef>
#include <cmath>
#include <cstdlib>
#include <cstring>
#include <functional>
#include <memory>
#include <mutex>
#include <numeric>
#include <string>
#include <vector>

#include "footprint.h"
#include "insitu_kernels.h"
#include "rt_ctx.h"
#include "rt_kernels.h"
#include "spray_rt.h"

using namespace spray_rt;
using namespace spray_rt::detail;

namespace {

// ---------------------------------------------------------------------------
// RCCL, resolved at run time: the copy already in the process (PyTorch's)
// when there is one, else the system's librccl.so.1 -- one RCCL per process.
// ---------------------------------------------------------------------------
struct NcclApi {
  bool ok = false;
  std::string err;
  ncclResult_t (*GetUniqueId)(ncclUniqueId*) = nullptr;
  ncclResult_t (*CommInitRank)(ncclComm_t*, int, ncclUniqueId, int) = nullptr;
  ncclResult_t (*CommDestroy)(ncclComm_t) = nullptr;
  ncclResult_t (*GroupStart)() = nullptr;
  ncclResult_t (*GroupEnd)() = nullptr;
  ncclResult_t (*Send)(const void*, size_t, ncclDataType_t, int, ncclComm_t, hipStream_t) = nullptr;
  ncclResult_t (*Recv)(void*, size_t, ncclDataType_t, int, ncclComm_t, hipStream_t) = nullptr;
  ncclResult_t (*AllReduce)(const void*, void*, size_t, ncclDataType_t, ncclRedOp_t, ncclComm_t,
                            hipStream_t) = nullptr;
  ncclResult_t (*Reduce)(const void*, void*, size_t, ncclDataType_t, ncclRedOp_t, int,
                         ncclComm_t, hipStream_t) = nullptr;
  const char* (*GetErrorString)(ncclResult_t) = nullptr;
};

NcclApi& nccl() {
  static NcclApi api;
  static std::once_flag once;
  std::call_once(once, [] {
    void* h = nullptr;
    for (const char* name : {"librccl.so", "librccl.so.1"})
      if ((h = dlopen(name, RTLD_NOW | RTLD_NOLOAD))) break;
    if (!h) h = dlopen("librccl.so.1", RTLD_NOW | RTLD_LOCAL);
    if (!h) h = dlopen("/opt/rocm/lib/librccl.so.1", RTLD_NOW | RTLD_LOCAL);
    if (!h) {
      api.err = std::string("cannot load librccl: ") + dlerror();
      return;
    }
    bool all = true;
    auto sym = [&](auto& fn, const char* name) {
      fn = reinterpret_cast<std::remove_reference_t<decltype(fn)>>(dlsym(h, name));
      all &= fn != nullptr;
    };
    sym(api.GetUniqueId, "ncclGetUniqueId");
    sym(api.CommInitRank, "ncclCommInitRank");
    sym(api.CommDestroy, "ncclCommDestroy");
    sym(api.GroupStart, "ncclGroupStart");
    sym(api.GroupEnd, "ncclGroupEnd");
    sym(api.Send, "ncclSend");
    sym(api.Recv, "ncclRecv");
    sym(api.AllReduce, "ncclAllReduce");
    sym(api.Reduce, "ncclReduce");
    sym(api.GetErrorString, "ncclGetErrorString");
    if (!all) {
      api.err = "librccl lacks a required entry point";
      return;
    }
    api.ok = true;
  });
  return api;
}

struct DBuf {
  void* p = nullptr;
  size_t cap = 0;
  template <typename T>
  T* as() const {
    return static_cast<T*>(p);
  }
};

}  // namespace

// ---------------------------------------------------------------------------
// transports
// ---------------------------------------------------------------------------
// The issue log of the group's collectives (spray_rt_insitu_collective_log):
// RCCL needs every rank to enqueue the same collectives in the same order
// (per communicator, across its streams), so each call is recorded as
// op << 56 | side stream << 51 | element count (48 bits) before it runs.
// The all-to-all-v's per-peer byte counts legitimately differ between ranks
// (they match pairwise), so those entries carry no count.
enum CollOp : uint64_t {
  kCollCounts = 1,        // int64[world] count all-to-all
  kCollAlltoallv = 2,     // bytes, per-peer counts
  kCollSumU64 = 3,        // all-reduce SUM u64
  kCollReduceF32 = 4,     // reduce SUM f32 to a root
  kCollMinU64 = 5,        // all-reduce MIN u64
  kCollSumU8 = 6,         // all-reduce SUM u8
  kCollMinU32 = 7,        // all-reduce MIN u32 (t bits)
  kCollMinU8 = 8,         // all-reduce MIN u8 (list positions)
};
void collective_log(spray_rt_insitu* I, uint64_t op, size_t n, hipStream_t st);

struct InsituTransport {
  virtual ~InsituTransport() = default;
  // per-peer counts: dev_send (device int64[world]) -> host send / recv
  int counts(spray_rt_insitu* I, const int64_t* dev_send, int64_t* h_send, int64_t* h_recv);
  // device buffers; byte counts per peer (host)
  // skip_self: the rank's own segment is not moved (its offsets still count)
  int alltoallv(spray_rt_insitu* I, const void* send, const size_t* sb, void* recv,
                const size_t* rb, bool skip_self = false);
  int allreduce_u64(spray_rt_insitu* I, unsigned long long* dev, size_t n);
  int reduce_f32(spray_rt_insitu* I, float* dev, size_t n, int root);
  // replicated-ray frames: MIN of u64 keys, SUM of bytes (device, in place)
  virtual bool has_rep() const { return true; }
  int allreduce_min_u64(spray_rt_insitu* I, uint64_t* dev, size_t n);
  int allreduce_sum_u8(spray_rt_insitu* I, uint8_t* dev, size_t n);
  // split keys: MIN of u32 t bits (src -> dst; in place when equal) and of
  // u8 list positions, on stream st (RCCL: overlapping the other streams'
  // work; the host form runs them in order, blocking); off = the slots'
  // first index in the frame's U (the replay's captured arrays)
  int allreduce_min_u32(spray_rt_insitu* I, const uint32_t* src, uint32_t* dst, size_t n,
                        size_t off, hipStream_t st);
  int allreduce_min_u8(spray_rt_insitu* I, uint8_t* dev, size_t n, size_t off, hipStream_t st);

 protected:
  // the transports' implementations of the calls above (which log first)
  virtual int do_counts(spray_rt_insitu* I, const int64_t* dev_send, int64_t* h_send,
                        int64_t* h_recv) = 0;
  virtual int do_alltoallv(spray_rt_insitu* I, const void* send, const size_t* sb, void* recv,
                           const size_t* rb, bool skip_self) = 0;
  virtual int do_allreduce_u64(spray_rt_insitu* I, unsigned long long* dev, size_t n) = 0;
  virtual int do_reduce_f32(spray_rt_insitu* I, float* dev, size_t n, int root) = 0;
  virtual int do_allreduce_min_u64(spray_rt_insitu* I, uint64_t* dev, size_t n) = 0;
  virtual int do_allreduce_sum_u8(spray_rt_insitu* I, uint8_t* dev, size_t n) = 0;
  virtual int do_allreduce_min_u32(spray_rt_insitu* I, const uint32_t* src, uint32_t* dst,
                                   size_t n, size_t off, hipStream_t st) = 0;
  virtual int do_allreduce_min_u8(spray_rt_insitu* I, uint8_t* dev, size_t n, size_t off,
                                  hipStream_t st) = 0;

 public:
  // rehearsal only: the rank's device work runs while it holds a lock
  // shared by the group's processes (SPRAY_INSITU_SERIAL), so the phase
  // timings of ranks sharing one GPU are not inflated by each other
  virtual void serial_begin() {}
  virtual void serial_end() {}
  // copies a rank sends itself may skip the wire (the owner gathers them
  // straight from the holder's arrays)
  virtual bool self_direct() const { return true; }
  // collectives enqueued on a side stream run beside the main stream's work
  // (RCCL); the host form runs them in order, blocking
  virtual bool side_stream() const { return false; }
};

struct spray_rt_insitu {
  spray_rt_ctx* ctx = nullptr;
  int world = 1, rank = 0;
  std::unique_ptr<InsituTransport> tr;
  // holder batch of the next bounce (double buffered)
  DBuf hray[2], hw[2], hpix[2], hsam[2];
  // routing / plan
  DBuf mask, idx, starts, plan_tmp, dcnt;
  // wire buffers
  DBuf sendb, recvb;
  // owner copies
  DBuf oray, ow, opix, osam, ohit, okey, obest, owin, ovalid;
  // holder side of the key composite
  DBuf best, keyback;
  // shadow slots of the shaded copies and their exchange
  DBuf sray, ssw, ssv, socc, ssel, smask, sidx, sstarts, ashadow, aocc, sret;
  DBuf nsel, sel_tmp, dnum, dstats, dtot;
  unsigned long long* h_small = nullptr;  // pinned: counts, totals
  unsigned long long st[6] = {0, 0, 0, 0, 0, 0};
  // replicated-ray frames (trace_replicated)
  DBuf rfc, ridx_c, rnum, rsel_tmp, rkeys_n, rhits_n, rkeys_c;
  DBuf rsray, rsflag, rwin, rsvalid, rsw, rocc, rpix, rsam, rhit_c, rnsh;
  // replicated-ray AO frames (trace_replicated_ao)
  DBuf apub, arays, ahits, apairs, aocc_p, alv, arec, ascratch, afields, acount;
  DBuf aflag, aown, asel_tmp;  // replicated AO: the own pairs, compacted
  DBuf abits;                  // their first round's occlusion, one bit per pair
  // compact film of replicated PT frames (runs of equal pixels along C)
  DBuf rincl, rscan_tmp, rslot_c, rslot_pix, rcompact, rnp;
  hipEvent_t ev_np = nullptr;  // the run count's copy to the host
  // split keys: t bits and list positions over C; the list positions'
  // all-reduce runs on a second stream (cs) beside the shadow any hit
  DBuf rtk, rlp, rbmax;
  // camera frames (trace_camera): the run tables of the last camera (U =
  // the pixels any box may be seen through; E / S = this rank's eye and
  // shadow footprints), their key, and the frame's arrays over U
  std::vector<float> cam_key;
  DBuf tu_runs, tu_first, te_runs, te_first, ts_runs, ts_first;
  CamTable tu{}, te{}, ts{};
  uint32_t tu_pixmax = 0;
  size_t last_nu = 0;     // U slots of the last camera PT frame
  size_t last_nc_ao = 0;  // C slots of the last replicated AO frame
  size_t last_npair_ao = 0;  // and its AO pairs (nc x samples)
  DBuf ctmin, ccomp, crays, cpix, csam, ciota;
  DBuf gpack;  // image frames: the rank's interleaved bands packed / the root's gather
  // image frames: the run table of U within this rank's bands (its eye
  // rays), its key, and U's pixel count over the whole image
  std::vector<float> img_key;
  DBuf ti_runs, ti_first;
  CamTable ti{};
  uint64_t img_upix = 0;
  // the compact gather: every rank's pixels of U (its table's npix), and on
  // rank 0 the table of the other ranks' U pixels in rank order
  std::vector<uint32_t> img_counts;
  DBuf tg_runs, tg_first;
  CamTable tg{};
  size_t ciota_n = 0;  // entries of ciota filled (0 .. n - 1)
  hipStream_t cs = nullptr;
  hipEvent_t ev_lp0 = nullptr, ev_lp1 = nullptr;
  // phase timing (spray_rt_insitu_set_timing): events on the stream
  bool timing = false;
  static constexpr int kMaxEv = 48;
  hipEvent_t ev[kMaxEv] = {};
  int ev_phase[kMaxEv] = {};
  int nev = 0, nph = 0, cur_phase = 0;
  double phase_ms[9] = {0, 0, 0, 0, 0, 0, 0, 0, 0};  // [8]: inside collectives
  // the collectives' issue log since the last read (CollOp entries; at most
  // kMaxLog kept, clog_total counts every one)
  static constexpr size_t kMaxLog = 1 << 16;
  std::vector<uint64_t> clog;
  uint64_t clog_total = 0;
};

void collective_log(spray_rt_insitu* I, uint64_t op, size_t n, hipStream_t st) {
  const uint64_t side = (st && st != stream_of(I->ctx)) ? 1 : 0;
  if (I->clog.size() < spray_rt_insitu::kMaxLog)
    I->clog.push_back(op << 56 | side << 51 | (uint64_t(n) & ((uint64_t(1) << 48) - 1)));
  ++I->clog_total;
}

int InsituTransport::counts(spray_rt_insitu* I, const int64_t* dev_send, int64_t* h_send,
                            int64_t* h_recv) {
  collective_log(I, kCollCounts, size_t(I->world), nullptr);
  return do_counts(I, dev_send, h_send, h_recv);
}
int InsituTransport::alltoallv(spray_rt_insitu* I, const void* send, const size_t* sb, void* recv,
                               const size_t* rb, bool skip_self) {
  collective_log(I, kCollAlltoallv, 0, nullptr);
  return do_alltoallv(I, send, sb, recv, rb, skip_self);
}
int InsituTransport::allreduce_u64(spray_rt_insitu* I, unsigned long long* dev, size_t n) {
  collective_log(I, kCollSumU64, n, nullptr);
  return do_allreduce_u64(I, dev, n);
}
int InsituTransport::reduce_f32(spray_rt_insitu* I, float* dev, size_t n, int root) {
  collective_log(I, kCollReduceF32, n, nullptr);
  return do_reduce_f32(I, dev, n, root);
}
int InsituTransport::allreduce_min_u64(spray_rt_insitu* I, uint64_t* dev, size_t n) {
  collective_log(I, kCollMinU64, n, nullptr);
  return do_allreduce_min_u64(I, dev, n);
}
int InsituTransport::allreduce_sum_u8(spray_rt_insitu* I, uint8_t* dev, size_t n) {
  collective_log(I, kCollSumU8, n, nullptr);
  return do_allreduce_sum_u8(I, dev, n);
}
int InsituTransport::allreduce_min_u32(spray_rt_insitu* I, const uint32_t* src, uint32_t* dst,
                                       size_t n, size_t off, hipStream_t st) {
  collective_log(I, kCollMinU32, n, st);
  return do_allreduce_min_u32(I, src, dst, n, off, st);
}
int InsituTransport::allreduce_min_u8(spray_rt_insitu* I, uint8_t* dev, size_t n, size_t off,
                                      hipStream_t st) {
  collective_log(I, kCollMinU8, n, st);
  return do_allreduce_min_u8(I, dev, n, off, st);
}

namespace {

int grow(spray_rt_insitu* I, DBuf& b, size_t bytes) {
  if (b.cap >= bytes) return SPRAY_RT_OK;
  spray_rt_ctx* c = I->ctx;
  if (b.p) {
    HIPCHK(c, hipStreamSynchronize(stream_of(c)));  // queued work may still read it
    HIPCHK(c, hipFree(b.p));
  }
  b.p = nullptr;
  b.cap = 0;
  const size_t want = std::max<size_t>(align256(bytes + bytes / 8), 4096);
  HIPCHK(c, hipMalloc(&b.p, want));
  b.cap = want;
  return SPRAY_RT_OK;
}

#define GROW(b, bytes)                          \
  do {                                          \
    int _r = grow(I, (b), (bytes));             \
    if (_r) return _r;                          \
  } while (0)
#define CALL(expr)                              \
  do {                                          \
    int _r = (expr);                            \
    if (_r) return _r;                          \
  } while (0)

// ---- RCCL ----
struct RcclTransport : InsituTransport {
  ncclComm_t comm = nullptr;
  bool self_via_nccl = false;  // route self traffic through ncclSend/Recv (tests)

  int chk(spray_rt_insitu* I, ncclResult_t r, const char* what) {
    if (r == ncclSuccess) return SPRAY_RT_OK;
    return fail(I->ctx, SPRAY_RT_ERR_HIP, "%s: %s", what, nccl().GetErrorString(r));
  }
  int do_counts(spray_rt_insitu* I, const int64_t* dev_send, int64_t* h_send,
             int64_t* h_recv) override {
    const int W = I->world;
    int64_t* dev_recv = const_cast<int64_t*>(dev_send) + 64;
    std::vector<size_t> b(W, sizeof(int64_t));
    CALL(do_alltoallv(I, dev_send, b.data(), dev_recv, b.data(), false));
    hipStream_t s = stream_of(I->ctx);
    HIPCHK(I->ctx, hipMemcpyAsync(I->h_small, dev_send, 128 * sizeof(int64_t),
                                  hipMemcpyDeviceToHost, s));
    HIPCHK(I->ctx, hipStreamSynchronize(s));
    std::memcpy(h_send, I->h_small, W * sizeof(int64_t));
    std::memcpy(h_recv, I->h_small + 64, W * sizeof(int64_t));
    ++I->st[3];
    return SPRAY_RT_OK;
  }
  int do_alltoallv(spray_rt_insitu* I, const void* send, const size_t* sb, void* recv,
                const size_t* rb, bool skip_self) override {
    const NcclApi& N = nccl();
    hipStream_t s = stream_of(I->ctx);
    const char* sp = static_cast<const char*>(send);
    char* rp = static_cast<char*>(recv);
    size_t so = 0, ro = 0;
    CALL(chk(I, N.GroupStart(), "ncclGroupStart"));
    for (int r = 0; r < I->world; ++r) {
      if (r == I->rank && !self_via_nccl) {
        if (sb[r] && !skip_self)
          HIPCHK(I->ctx, hipMemcpyAsync(rp + ro, sp + so, sb[r], hipMemcpyDeviceToDevice, s));
      } else {
        if (sb[r]) CALL(chk(I, N.Send(sp + so, sb[r], ncclUint8, r, comm, s), "ncclSend"));
        if (rb[r]) CALL(chk(I, N.Recv(rp + ro, rb[r], ncclUint8, r, comm, s), "ncclRecv"));
      }
      so += sb[r];
      ro += rb[r];
    }
    CALL(chk(I, N.GroupEnd(), "ncclGroupEnd"));
    ++I->st[4];
    return SPRAY_RT_OK;
  }
  int do_allreduce_u64(spray_rt_insitu* I, unsigned long long* dev, size_t n) override {
    ++I->st[4];
    return chk(I, nccl().AllReduce(dev, dev, n, ncclUint64, ncclSum, comm, stream_of(I->ctx)),
               "ncclAllReduce");
  }
  int do_reduce_f32(spray_rt_insitu* I, float* dev, size_t n, int root) override {
    ++I->st[4];
    return chk(I, nccl().Reduce(dev, dev, n, ncclFloat32, ncclSum, root, comm, stream_of(I->ctx)),
               "ncclReduce");
  }
  int do_allreduce_min_u64(spray_rt_insitu* I, uint64_t* dev, size_t n) override {
    ++I->st[4];
    return chk(I, nccl().AllReduce(dev, dev, n, ncclUint64, ncclMin, comm, stream_of(I->ctx)),
               "ncclAllReduce(min)");
  }
  int do_allreduce_sum_u8(spray_rt_insitu* I, uint8_t* dev, size_t n) override {
    ++I->st[4];
    return chk(I, nccl().AllReduce(dev, dev, n, ncclUint8, ncclSum, comm, stream_of(I->ctx)),
               "ncclAllReduce(sum u8)");
  }
  int do_allreduce_min_u32(spray_rt_insitu* I, const uint32_t* src, uint32_t* dst, size_t n,
                        size_t, hipStream_t st) override {
    ++I->st[4];
    return chk(I, nccl().AllReduce(src, dst, n, ncclUint32, ncclMin, comm, st),
               "ncclAllReduce(min u32)");
  }
  int do_allreduce_min_u8(spray_rt_insitu* I, uint8_t* dev, size_t n, size_t,
                       hipStream_t st) override {
    ++I->st[4];
    return chk(I, nccl().AllReduce(dev, dev, n, ncclUint8, ncclMin, comm, st),
               "ncclAllReduce(min u8)");
  }
  bool self_direct() const override { return !self_via_nccl; }
  bool side_stream() const override { return true; }
  ~RcclTransport() override {
    if (comm) nccl().CommDestroy(comm);
  }
};

// ---- replay (measurement: one rank of an N-rank group alone on one GPU) ----
// The group results of a camera frame given up front (the t-bits and
// list-position MINs over U, captured from a one-rank frame with every
// domain resident): the MINs copy them, the SUMs and the reduce keep the
// rank's own values.  The rank's device work is then its exact share of the
// N-rank frame, back to back on its stream with no idle gaps between
// collectives (the per-rank segment times of the multi-GPU projection).
struct ReplayTransport : InsituTransport {
  const uint32_t* tmin = nullptr;
  const uint8_t* lpmin = nullptr;
  size_t n = 0;
  // AO camera frames: the key MIN over U and the published winners'
  // normals and colours (the SUM of the publish step, 16 B per slot)
  const uint64_t* kmin = nullptr;
  const uint64_t* pub = nullptr;
  size_t nk = 0;
  // and the first round's occlusion bits of the group (the SUM of that
  // many bytes); other SUMs keep the rank's own values
  const uint8_t* bits = nullptr;
  size_t nbits_bytes = 0;
  int copy(spray_rt_insitu* I, void* dst, const void* src, size_t bytes, hipStream_t s) {
    ++I->st[4];
    if (bytes) HIPCHK(I->ctx, hipMemcpyAsync(dst, src, bytes, hipMemcpyDeviceToDevice, s));
    return SPRAY_RT_OK;
  }
  int need(spray_rt_insitu* I, size_t m, size_t off) {
    if (!tmin || off + m > n || I->last_nu != n)
      return fail(I->ctx, SPRAY_RT_ERR_STATE, "replay: %zu slots given, the frame has %zu", n,
                  I->last_nu);
    return SPRAY_RT_OK;
  }
  int do_counts(spray_rt_insitu* I, const int64_t*, int64_t*, int64_t*) override {
    return fail(I->ctx, SPRAY_RT_ERR_UNSUPPORTED, "replay transport: camera frames only");
  }
  // only the image frame's row gather reaches here (the protocol stops at
  // its count exchange above): the rank keeps its own rows
  int do_alltoallv(spray_rt_insitu* I, const void*, const size_t*, void*, const size_t*,
                   bool) override {
    ++I->st[4];
    return SPRAY_RT_OK;
  }
  int do_allreduce_u64(spray_rt_insitu* I, unsigned long long* dev, size_t m) override {
    if (!pub) {  // keep the rank's own values
      ++I->st[4];
      return SPRAY_RT_OK;
    }
    if (m != 2 * nk) return fail(I->ctx, SPRAY_RT_ERR_STATE, "replay: %zu publish words given, "
                                 "the frame has %zu", 2 * nk, m);
    return copy(I, dev, pub, m * 8, stream_of(I->ctx));
  }
  int do_reduce_f32(spray_rt_insitu* I, float*, size_t, int) override {
    ++I->st[4];
    return SPRAY_RT_OK;
  }
  int do_allreduce_min_u64(spray_rt_insitu* I, uint64_t* dev, size_t m) override {
    if (!kmin || m != nk)
      return fail(I->ctx, SPRAY_RT_ERR_STATE, "replay: %zu keys given, the frame has %zu", nk, m);
    return copy(I, dev, kmin, m * 8, stream_of(I->ctx));
  }
  int do_allreduce_sum_u8(spray_rt_insitu* I, uint8_t* dev, size_t m) override {
    if (bits && m == nbits_bytes) return copy(I, dev, bits, m, stream_of(I->ctx));
    ++I->st[4];
    return SPRAY_RT_OK;
  }
  int do_allreduce_min_u32(spray_rt_insitu* I, const uint32_t*, uint32_t* dst, size_t m,
                        size_t off, hipStream_t st) override {
    CALL(need(I, m, off));
    return copy(I, dst, tmin + off, m * 4, st);
  }
  int do_allreduce_min_u8(spray_rt_insitu* I, uint8_t* dev, size_t m, size_t off,
                       hipStream_t st) override {
    CALL(need(I, m, off));
    return copy(I, dev, lpmin + off, m, st);
  }
  bool side_stream() const override { return true; }
};

// ---- host callbacks (staged) ----
struct HostTransport : InsituTransport {
  spray_rt_transport cb{};
  std::vector<char> hs, hr;
  int lock_fd = -1;  // SPRAY_INSITU_SERIAL: the group's device-work lock

  ~HostTransport() override {
    if (lock_fd >= 0) close(lock_fd);
  }
  void serial_begin() override {
    if (lock_fd >= 0) (void)flock(lock_fd, LOCK_EX);
  }
  void serial_end() override {
    if (lock_fd >= 0) (void)flock(lock_fd, LOCK_UN);
  }
  // every collective first drains the stream (the staging below does), then
  // lets the other ranks' device work run while this one waits
  int sync(spray_rt_insitu* I) {
    HIPCHK(I->ctx, hipStreamSynchronize(stream_of(I->ctx)));
    return SPRAY_RT_OK;
  }
  bool has_rep() const override { return cb.allreduce_min_u64 && cb.allreduce_sum_u8; }
  int do_allreduce_min_u64(spray_rt_insitu* I, uint64_t* dev, size_t n) override {
    std::vector<unsigned long long> h(std::max<size_t>(n, 1));
    HIPCHK(I->ctx, hipMemcpyAsync(h.data(), dev, n * 8, hipMemcpyDeviceToHost, stream_of(I->ctx)));
    CALL(sync(I));
    serial_end();
    const int bad = cb.allreduce_min_u64(cb.user, h.data(), n);
    serial_begin();
    if (bad) return fail(I->ctx, SPRAY_RT_ERR_STATE, "host transport: min all-reduce failed");
    HIPCHK(I->ctx, hipMemcpyAsync(dev, h.data(), n * 8, hipMemcpyHostToDevice, stream_of(I->ctx)));
    CALL(sync(I));
    ++I->st[4];
    return SPRAY_RT_OK;
  }
  int do_allreduce_sum_u8(spray_rt_insitu* I, uint8_t* dev, size_t n) override {
    std::vector<uint8_t> h(std::max<size_t>(n, 1));
    HIPCHK(I->ctx, hipMemcpyAsync(h.data(), dev, n, hipMemcpyDeviceToHost, stream_of(I->ctx)));
    CALL(sync(I));
    serial_end();
    const int bad = cb.allreduce_sum_u8(cb.user, h.data(), n);
    serial_begin();
    if (bad) return fail(I->ctx, SPRAY_RT_ERR_STATE, "host transport: byte all-reduce failed");
    HIPCHK(I->ctx, hipMemcpyAsync(dev, h.data(), n, hipMemcpyHostToDevice, stream_of(I->ctx)));
    CALL(sync(I));
    ++I->st[4];
    return SPRAY_RT_OK;
  }
  // the narrow MINs through the 64-bit host callback (widened on the host),
  // staged on the stream that produced them
  template <typename T>
  int min_widened(spray_rt_insitu* I, T* dev, size_t n, hipStream_t st) {
    std::vector<T> h(std::max<size_t>(n, 1));
    std::vector<unsigned long long> w(std::max<size_t>(n, 1));
    HIPCHK(I->ctx, hipMemcpyAsync(h.data(), dev, n * sizeof(T), hipMemcpyDeviceToHost, st));
    HIPCHK(I->ctx, hipStreamSynchronize(st));
    for (size_t k = 0; k < n; ++k) w[k] = h[k];
    serial_end();
    const int bad = cb.allreduce_min_u64(cb.user, w.data(), n);
    serial_begin();
    if (bad) return fail(I->ctx, SPRAY_RT_ERR_STATE, "host transport: min all-reduce failed");
    for (size_t k = 0; k < n; ++k) h[k] = T(w[k]);
    HIPCHK(I->ctx, hipMemcpyAsync(dev, h.data(), n * sizeof(T), hipMemcpyHostToDevice, st));
    HIPCHK(I->ctx, hipStreamSynchronize(st));
    ++I->st[4];
    return SPRAY_RT_OK;
  }
  int do_allreduce_min_u32(spray_rt_insitu* I, const uint32_t* src, uint32_t* dst, size_t n,
                        size_t, hipStream_t st) override {
    if (src != dst && n)
      HIPCHK(I->ctx, hipMemcpyAsync(dst, src, n * 4, hipMemcpyDeviceToDevice, st));
    return min_widened(I, dst, n, st);
  }
  int do_allreduce_min_u8(spray_rt_insitu* I, uint8_t* dev, size_t n, size_t,
                       hipStream_t st) override {
    return min_widened(I, dev, n, st);
  }
  int do_counts(spray_rt_insitu* I, const int64_t* dev_send, int64_t* h_send,
             int64_t* h_recv) override {
    const int W = I->world;
    HIPCHK(I->ctx, hipMemcpyAsync(h_send, dev_send, W * sizeof(int64_t), hipMemcpyDeviceToHost,
                                  stream_of(I->ctx)));
    CALL(sync(I));
    std::vector<size_t> b(W, sizeof(int64_t));
    serial_end();
    const int bad = cb.alltoallv(cb.user, h_send, b.data(), h_recv, b.data());
    serial_begin();
    if (bad) return fail(I->ctx, SPRAY_RT_ERR_STATE, "host transport: count exchange failed");
    ++I->st[3];
    ++I->st[4];
    return SPRAY_RT_OK;
  }
  int do_alltoallv(spray_rt_insitu* I, const void* send, const size_t* sb, void* recv,
                const size_t* rb, bool) override {  // the self segment travels (unused)
    const int W = I->world;
    const size_t ts = std::accumulate(sb, sb + W, size_t(0));
    const size_t trv = std::accumulate(rb, rb + W, size_t(0));
    hs.resize(std::max<size_t>(ts, 1));
    hr.resize(std::max<size_t>(trv, 1));
    hipStream_t s = stream_of(I->ctx);
    if (ts) HIPCHK(I->ctx, hipMemcpyAsync(hs.data(), send, ts, hipMemcpyDeviceToHost, s));
    CALL(sync(I));
    serial_end();
    const int bad = cb.alltoallv(cb.user, hs.data(), sb, hr.data(), rb);
    serial_begin();
    if (bad) return fail(I->ctx, SPRAY_RT_ERR_STATE, "host transport: all-to-all failed");
    if (trv) HIPCHK(I->ctx, hipMemcpyAsync(recv, hr.data(), trv, hipMemcpyHostToDevice, s));
    CALL(sync(I));  // hr is reused by the next call
    ++I->st[4];
    return SPRAY_RT_OK;
  }
  int do_allreduce_u64(spray_rt_insitu* I, unsigned long long* dev, size_t n) override {
    std::vector<unsigned long long> h(n);
    HIPCHK(I->ctx, hipMemcpyAsync(h.data(), dev, n * 8, hipMemcpyDeviceToHost, stream_of(I->ctx)));
    CALL(sync(I));
    serial_end();
    const int bad = cb.allreduce_u64(cb.user, h.data(), n);
    serial_begin();
    if (bad) return fail(I->ctx, SPRAY_RT_ERR_STATE, "host transport: all-reduce failed");
    HIPCHK(I->ctx, hipMemcpyAsync(dev, h.data(), n * 8, hipMemcpyHostToDevice, stream_of(I->ctx)));
    CALL(sync(I));
    ++I->st[4];
    return SPRAY_RT_OK;
  }
  int do_reduce_f32(spray_rt_insitu* I, float* dev, size_t n, int root) override {
    std::vector<float> h(n);
    HIPCHK(I->ctx, hipMemcpyAsync(h.data(), dev, n * 4, hipMemcpyDeviceToHost, stream_of(I->ctx)));
    CALL(sync(I));
    serial_end();
    const int bad = cb.reduce_f32(cb.user, h.data(), n, root);
    serial_begin();
    if (bad) return fail(I->ctx, SPRAY_RT_ERR_STATE, "host transport: reduce failed");
    if (I->rank == root)
      HIPCHK(I->ctx, hipMemcpyAsync(dev, h.data(), n * 4, hipMemcpyHostToDevice, stream_of(I->ctx)));
    CALL(sync(I));
    ++I->st[4];
    return SPRAY_RT_OK;
  }
};

// One routed exchange: per-destination lists of a batch (route + plan), the
// count exchange (one host read), the per-peer byte counts.
struct Routed {
  size_t total = 0;  // copies this rank sends (entries of idx)
  size_t recv = 0;   // copies it receives
  size_t self_n = 0, self_send = 0, self_recv = 0;  // its own copies, their offsets
  std::vector<int64_t> send_n, recv_n;
  std::vector<size_t> bytes(size_t per, bool back) const {
    const std::vector<int64_t>& v = back ? recv_n : send_n;
    std::vector<size_t> b(v.size());
    for (size_t r = 0; r < v.size(); ++r) b[r] = size_t(v[r]) * per;
    return b;
  }
};

// ---- phase timing: an event at each phase start; the time to the next
// event is charged to that phase (read after the trace's last sync).  The
// time inside collectives (and the host reads they imply) goes to its own
// slot, kCommPhase, so the phases are the device work around them.
constexpr int kCommPhase = 8;
int mark(spray_rt_insitu* I, int phase) {
  if (phase != kCommPhase) I->cur_phase = phase;
  if (!I->timing || I->nev >= spray_rt_insitu::kMaxEv) return SPRAY_RT_OK;
  hipEvent_t& e = I->ev[I->nev];
  if (!e) HIPCHK(I->ctx, hipEventCreate(&e));
  HIPCHK(I->ctx, hipEventRecord(e, stream_of(I->ctx)));
  I->ev_phase[I->nev++] = phase;
  return SPRAY_RT_OK;
}
void flush_phases(spray_rt_insitu* I, int nphases) {
  if (!I->timing) return;
  for (int k = 0; k + 1 < I->nev; ++k) {
    float ms = 0.f;
    if (hipEventElapsedTime(&ms, I->ev[k], I->ev[k + 1]) == hipSuccess)
      I->phase_ms[I->ev_phase[k]] += double(ms);
  }
  I->nev = 0;
  I->nph = nphases;
}
#define MARK(ph) CALL(mark(I, (ph)))
// a collective: its stream time to kCommPhase, then back to the phase
#define COMM(expr)                    \
  do {                                \
    const int _ph = I->cur_phase;     \
    MARK(kCommPhase);                 \
    CALL(expr);                       \
    MARK(_ph);                        \
  } while (0)

int route_and_count(spray_rt_insitu* I, const spray_rt_ray* rays, size_t n, DBuf& mask, DBuf& idx,
                    DBuf& starts, Routed* R, const uint32_t* sel = nullptr,
                    const uint8_t* valid = nullptr) {
  spray_rt_ctx* c = I->ctx;
  hipStream_t s = stream_of(c);
  const int W = I->world;
  GROW(mask, n * 8);
  GROW(idx, n * size_t(W) * 8);
  GROW(starts, (W + 1) * 8);
  GROW(I->plan_tmp, plan_temp_bytes(n, W));
  GROW(I->dcnt, 128 * 8);
  if (n) HIPCHK(c, launch_route(s, view(c), c->d_owner, rays, n, mask.as<uint64_t>(), sel, valid));
  HIPCHK(c, launch_plan(s, mask.as<uint64_t>(), n, W, idx.as<int64_t>(), starts.as<int64_t>(),
                        I->plan_tmp.p));
  HIPCHK(c, launch_counts_from_starts(s, starts.as<int64_t>(), W, I->dcnt.as<int64_t>()));
  R->send_n.assign(W, 0);
  R->recv_n.assign(W, 0);
  COMM(I->tr->counts(I, I->dcnt.as<int64_t>(), R->send_n.data(), R->recv_n.data()));
  R->total = R->recv = 0;
  for (int r = 0; r < W; ++r) {
    if (R->send_n[r] < 0 || R->recv_n[r] < 0)
      return fail(c, SPRAY_RT_ERR_STATE, "in-situ count exchange returned a negative count");
    if (r == I->rank) {
      R->self_n = size_t(R->send_n[r]);
      R->self_send = R->total;
      R->self_recv = R->recv;
    }
    R->total += size_t(R->send_n[r]);
    R->recv += size_t(R->recv_n[r]);
  }
  ++I->st[2];
  return SPRAY_RT_OK;
}

int exchange(spray_rt_insitu* I, const Routed& R, size_t per, bool back, const void* send,
             void* recv, bool skip_self = false) {
  const std::vector<size_t> sb = R.bytes(per, back), rb = R.bytes(per, !back);
  for (int r = 0; r < I->world; ++r)
    if (r != I->rank) {
      I->st[0] += sb[r];
      I->st[1] += rb[r];
    }
  COMM(I->tr->alltoallv(I, send, sb.data(), recv, rb.data(), skip_self));
  return SPRAY_RT_OK;
}

int trace(spray_rt_insitu* I, const spray_rt_shader* P, const spray_rt_ray* rays,
          const int32_t* pixid, const int32_t* samid, size_t n, int spp, float* image,
          const spray_rt_insitu_rec* rec, unsigned long long totals[3]) {
  spray_rt_ctx* c = I->ctx;
  hipStream_t s = stream_of(c);
  const int ns = spray_rt_shadow_slots(P);
  const double scale = 1.0 / double(spp);
  GROW(I->dstats, 4 * 8);
  GROW(I->dtot, 4 * 8);
  GROW(I->dnum, 2 * 4);
  HIPCHK(c, hipMemsetAsync(I->dstats.p, 0, 4 * 8, s));
  // bounce 0: the caller's eye rays, path weights (1, 1, 1)
  const spray_rt_ray* hr = rays;
  const int32_t* hp = pixid;
  const int32_t* hs = samid;
  const float* hw = nullptr;  // bounce 0: the packers write weights (1, 1, 1)
  size_t hn = n;
  int cur = 0;
  unsigned long long nrad = 0;
  for (int b = 0; b < P->bounces; ++b) {
    nrad += hn;
    // ---- radiance rays to the owners of their domains
    MARK(0);
    Routed R;
    CALL(route_and_count(I, hr, hn, I->mask, I->idx, I->starts, &R));
    MARK(1);
    const size_t m = R.recv;
    GROW(I->sendb, std::max(R.total * kRadRecBytes, R.total * 8));
    GROW(I->recvb, m * kRadRecBytes);
    // the rank's own copies skip the wire: the owner side gathers them from
    // the holder arrays (same records, same positions)
    const bool direct = I->tr->self_direct() && R.self_n;
    const size_t ps = direct ? R.self_send : R.total, pe = direct ? R.self_send + R.self_n : R.total;
    const size_t us = direct ? R.self_recv : m, ue = direct ? R.self_recv + R.self_n : m;
    char* sbp = static_cast<char*>(I->sendb.p);
    char* rbp = static_cast<char*>(I->recvb.p);
    const int64_t* ix = I->idx.as<int64_t>();
    HIPCHK(c, launch_pack_rad(s, hr, hw, hp, hs, ix, ps, sbp));
    HIPCHK(c, launch_pack_rad(s, hr, hw, hp, hs, ix + pe, R.total - pe, sbp + pe * kRadRecBytes));
    CALL(exchange(I, R, kRadRecBytes, false, I->sendb.p, I->recvb.p, direct));
    GROW(I->oray, m * 32);
    GROW(I->ow, m * 16);
    GROW(I->opix, m * 4);
    GROW(I->osam, m * 4);
    GROW(I->ohit, m * 48);
    GROW(I->okey, m * 8);
    GROW(I->obest, m * 8);
    GROW(I->owin, m);
    GROW(I->ovalid, m);
    spray_rt_ray* oray = I->oray.as<spray_rt_ray>();
    float* ow = I->ow.as<float>();
    int32_t* opix = I->opix.as<int32_t>();
    int32_t* osam = I->osam.as<int32_t>();
    HIPCHK(c, launch_unpack_rad(s, rbp, us, oray, ow, opix, osam));
    HIPCHK(c, launch_unpack_rad(s, rbp + ue * kRadRecBytes, m - ue, oray + ue, ow + 4 * ue,
                                opix + ue, osam + ue));
    if (direct)
      HIPCHK(c, launch_gather_rad(s, hr, hw, hp, hs, ix + R.self_send, R.self_n, oray + us,
                                  ow + 4 * us, opix + us, osam + us));
    MARK(2);
    if (m)
      HIPCHK(c, launch_scene_intersect_keyed(s, view(c), I->oray.as<spray_rt_ray>(), m,
                                             I->ohit.as<spray_rt_hit>(), I->okey.as<uint64_t>()));
    // ---- keys back to the holder, minimum per ray, the minimum forward
    MARK(3);
    GROW(I->keyback, R.total * 8);
    GROW(I->best, hn * 8);
    CALL(exchange(I, R, 8, true, I->okey.p, I->keyback.p));
    HIPCHK(c, launch_fill_u64(s, I->best.as<uint64_t>(), hn, kInsituMissKey));
    HIPCHK(c, launch_key_min(s, I->idx.as<int64_t>(), I->keyback.as<uint64_t>(), R.total,
                             I->best.as<uint64_t>()));
    if (R.total)
      HIPCHK(c, launch_gather_rows(s, I->best.p, 8, I->idx.as<int64_t>(), R.total, I->sendb.p));
    CALL(exchange(I, R, 8, false, I->sendb.p, I->obest.p));
    HIPCHK(c, launch_winners(s, I->okey.as<uint64_t>(), I->obest.as<uint64_t>(), m,
                             I->owin.as<uint8_t>()));
    // ---- the winning owner shades (ShaderPt / ShaderAo at ray depth b)
    MARK(4);
    const size_t MS = m * size_t(ns);
    if (m > 0xFFFFFFFFull || MS > 0xFFFFFFFFull)
      return fail(c, SPRAY_RT_ERR_LIMIT, "in-situ batch too large (copies x shadow slots > 2^32)");
    GROW(I->sray, MS * 32);
    GROW(I->ssw, MS * 16);
    GROW(I->ssv, MS);
    GROW(I->socc, MS);
    if (m) HIPCHK(c, hipMemcpyAsync(I->ovalid.p, I->owin.p, m, hipMemcpyDeviceToDevice, s));
    HIPCHK(c, launch_shade(s, *P, c->d_bsdf, c->nbsdf, b, ns, I->oray.as<spray_rt_ray>(),
                           I->ohit.as<spray_rt_hit>(), I->ow.as<float>(), I->ovalid.as<uint8_t>(),
                           I->opix.as<int32_t>(), I->osam.as<int32_t>(), m,
                           I->sray.as<spray_rt_ray>(), I->ssw.as<float>(), I->ssv.as<uint8_t>(),
                           I->dstats.as<unsigned long long>(), 1));
    // ---- shadow slots and next radiance rays.  One shadow slot per copy
    // (PT): the slots are routed in place, invalid ones owning no rank -- no
    // compaction and no host read.  Several (AO): compacted first (the
    // count is read); so are the next bounce's radiance rays.
    const bool more = b + 1 < P->bounces;
    const bool slots_direct = ns == 1;
    size_t cs = 0, cn = 0;
    if (!slots_direct || more) {
      size_t t1 = 0, t2 = 0;
      HIPCHK(c, launch_select_flagged(s, nullptr, MS, nullptr, nullptr, nullptr, &t1));
      HIPCHK(c, launch_select_flagged(s, nullptr, m, nullptr, nullptr, nullptr, &t2));
      GROW(I->sel_tmp, std::max(t1, t2));
      GROW(I->ssel, MS * 4);
      GROW(I->nsel, m * 4);
      uint32_t* dnum = I->dnum.as<uint32_t>();
      if (!slots_direct)
        HIPCHK(c, launch_select_flagged(s, I->ssv.as<uint8_t>(), MS, I->ssel.as<uint32_t>(), dnum,
                                        I->sel_tmp.p, &t1));
      else
        HIPCHK(c, hipMemsetAsync(dnum, 0, 4, s));
      if (more)
        HIPCHK(c, launch_select_flagged(s, I->ovalid.as<uint8_t>(), m, I->nsel.as<uint32_t>(),
                                        dnum + 1, I->sel_tmp.p, &t2));
      else
        HIPCHK(c, hipMemsetAsync(dnum + 1, 0, 4, s));
      HIPCHK(c, hipMemcpyAsync(I->h_small, dnum, 8, hipMemcpyDeviceToHost, s));
      HIPCHK(c, hipStreamSynchronize(s));
      ++I->st[3];
      uint32_t cnt2[2];
      std::memcpy(cnt2, I->h_small, 8);
      cs = cnt2[0];
      cn = cnt2[1];
    }
    // ---- shadow rays to the owners of their domains, occlusion OR-ed back
    MARK(5);
    if (MS) HIPCHK(c, hipMemsetAsync(I->socc.p, 0, MS, s));
    Routed S;  // the shadow rays, read in place (through ssel when compacted)
    const uint32_t* ssel = slots_direct ? nullptr : I->ssel.as<uint32_t>();
    if (slots_direct)
      CALL(route_and_count(I, I->sray.as<spray_rt_ray>(), MS, I->smask, I->sidx, I->sstarts, &S,
                           nullptr, I->ssv.as<uint8_t>()));
    else
      CALL(route_and_count(I, I->sray.as<spray_rt_ray>(), cs, I->smask, I->sidx, I->sstarts, &S,
                           ssel));
    GROW(I->sendb, S.total * kShadowRecBytes);
    GROW(I->recvb, S.recv * kShadowRecBytes);
    {
      const bool sdir = I->tr->self_direct() && S.self_n;
      const size_t a0 = sdir ? S.self_send : S.total, a1 = sdir ? S.self_send + S.self_n : S.total;
      const size_t b0 = sdir ? S.self_recv : S.recv, b1 = sdir ? S.self_recv + S.self_n : S.recv;
      const spray_rt_ray* sr = I->sray.as<spray_rt_ray>();
      const int64_t* six = I->sidx.as<int64_t>();
      char* sbp = static_cast<char*>(I->sendb.p);
      char* rbp = static_cast<char*>(I->recvb.p);
      HIPCHK(c, launch_pack_shadow(s, sr, ssel, six, a0, sbp));
      HIPCHK(c, launch_pack_shadow(s, sr, ssel, six + a1, S.total - a1, sbp + a1 * kShadowRecBytes));
      CALL(exchange(I, S, kShadowRecBytes, false, I->sendb.p, I->recvb.p, sdir));
      GROW(I->ashadow, S.recv * 32);
      GROW(I->aocc, S.recv);
      GROW(I->sret, S.total);
      spray_rt_ray* ash = I->ashadow.as<spray_rt_ray>();
      HIPCHK(c, launch_unpack_shadow(s, rbp, b0, ash));
      HIPCHK(c, launch_unpack_shadow(s, rbp + b1 * kShadowRecBytes, S.recv - b1, ash + b1));
      if (sdir)
        HIPCHK(c, launch_gather_shadow_self(s, sr, ssel, six + S.self_send, S.self_n, ash + b0));
    }
    MARK(6);
    if (S.recv)
      HIPCHK(c, launch_scene_occluded(s, view(c), I->ashadow.as<spray_rt_ray>(), S.recv, nullptr,
                                      I->aocc.as<uint8_t>(), nullptr));
    CALL(exchange(I, S, 1, true, I->aocc.p, I->sret.p));
    HIPCHK(c, launch_occ_return(s, I->sidx.as<int64_t>(), I->sret.as<uint8_t>(), S.total, ssel,
                                I->socc.as<uint8_t>()));
    // ---- film of the copies this rank shaded
    MARK(7);
    HIPCHK(c, launch_film_atomic(s, image, I->opix.as<int32_t>(), m, ns, I->ssw.as<float>(),
                                 I->ssv.as<uint8_t>(), I->socc.as<uint8_t>(), scale));
    if (rec)
      HIPCHK(c, launch_record(s, I->owin.as<uint8_t>(), m, b, ns, I->osam.as<int32_t>(),
                              I->ohit.as<spray_rt_hit>(), I->ssv.as<uint8_t>(),
                              I->socc.as<uint8_t>(), *rec));
    // ---- the spawned radiance rays: this rank's batch of the next bounce
    if (more) {
      const int nx = cur ^ 1;
      GROW(I->hray[nx], cn * 32);
      GROW(I->hw[nx], cn * 16);
      GROW(I->hpix[nx], cn * 4);
      GROW(I->hsam[nx], cn * 4);
      HIPCHK(c, launch_gather_next(s, I->oray.as<spray_rt_ray>(), I->ow.as<float>(),
                                   I->opix.as<int32_t>(), I->osam.as<int32_t>(),
                                   I->nsel.as<uint32_t>(), cn, I->hray[nx].as<spray_rt_ray>(),
                                   I->hw[nx].as<float>(), I->hpix[nx].as<int32_t>(),
                                   I->hsam[nx].as<int32_t>()));
      cur = nx;
      hr = I->hray[cur].as<spray_rt_ray>();
      hw = I->hw[cur].as<float>();
      hp = I->hpix[cur].as<int32_t>();
      hs = I->hsam[cur].as<int32_t>();
      hn = cn;
    }
  }
  // ---- the group's totals (WorkStats-like: one small all-reduce)
  // rays from the host's counts, shadows and aborts from the device's
  // shading counters: staged without a round trip, one all-reduce, one read
  // (h_small[0, 128) holds the count exchanges; every earlier use of these
  // two slots finished at this trace's last host read)
  unsigned long long* hin = I->h_small + 192;  // read by the queued copy
  unsigned long long* ht = I->h_small + 200;
  hin[0] = nrad;
  HIPCHK(c, hipMemcpyAsync(I->dtot.p, hin, 8, hipMemcpyHostToDevice, s));
  HIPCHK(c, hipMemcpyAsync(I->dtot.as<unsigned long long>() + 1,
                           I->dstats.as<unsigned long long>() + 1, 8, hipMemcpyDeviceToDevice, s));
  HIPCHK(c, hipMemcpyAsync(I->dtot.as<unsigned long long>() + 2, I->dstats.p, 8,
                           hipMemcpyDeviceToDevice, s));
  COMM(I->tr->allreduce_u64(I, I->dtot.as<unsigned long long>(), 3));
  HIPCHK(c, hipMemcpyAsync(ht, I->dtot.p, 3 * 8, hipMemcpyDeviceToHost, s));
  MARK(7);
  HIPCHK(c, hipStreamSynchronize(s));
  flush_phases(I, 8);
  if (totals)
    for (int k = 0; k < 3; ++k) totals[k] = ht[k];
  ++I->st[5];
  if (ht[2])
    return fail(c, SPRAY_RT_ERR_UNSUPPORTED, "%llu shading cases the reference aborts on", ht[2]);
  return SPRAY_RT_OK;
}

// Every domain is this rank's (one rank, or a partition that gives it all
// of them): no copy of any ray can leave the rank and every ray's only
// owner is its holder, so the exchange plans, the count reads and the key
// round trip have nothing to decide.  The frame then runs as the device
// frame layer does on the holder's own slots: per bounce closest hit over
// the whole domain list, shading, any hit of the shadow slots, film --
// with a single-point-light PT bounce as ONE fused launch (closest hit +
// shading + the shadow rays' any hit, launch_scene_frame_pt).  Results per
// sample are the protocol's (the same winner, shading and occlusion); the
// film adds with the same atomics; the totals come from the shading
// counters on the device and go through the transport's all-reduce.
//
// Only a one-rank group decides this alone.  With world > 1, a rank that owns
// every domain cannot tell from its owner map that the others hold no rays:
// they still route theirs to it through the count exchange, so every rank
// must run the same collectives (trace) -- a rank-local shortcut there would
// pair an all-reduce with the others' all-to-all and hang the group.
bool all_local(const spray_rt_insitu* I) { return I->world == 1; }

int trace_local(spray_rt_insitu* I, const spray_rt_shader* P, const spray_rt_ray* rays,
                const int32_t* pixid, const int32_t* samid, size_t n, int spp, float* image,
                const spray_rt_insitu_rec* rec, unsigned long long totals[3],
                const std::function<int()>& before_totals = {}) {
  spray_rt_ctx* c = I->ctx;
  hipStream_t s = stream_of(c);
  const int ns = spray_rt_shadow_slots(P);
  const size_t MS = n * size_t(ns);
  if (MS > 0xFFFFFFFFull) return fail(c, SPRAY_RT_ERR_LIMIT, "in-situ batch too large");
  const double scale = 1.0 / double(spp);
  GROW(I->dstats, 4 * 8);
  GROW(I->dtot, 4 * 8);
  GROW(I->dnum, 2 * 4);
  GROW(I->ohit, n * 48);
  GROW(I->owin, n);
  GROW(I->sray, MS * 32);
  GROW(I->ssw, MS * 16);
  GROW(I->ssv, MS);
  GROW(I->socc, MS);
  MARK(0);
  unsigned long long* st = I->dstats.as<unsigned long long>();
  unsigned long long* dt = I->dtot.as<unsigned long long>();
  spray_rt_hit* hits = I->ohit.as<spray_rt_hit>();
  uint8_t* sv = I->ssv.as<uint8_t>();
  uint8_t* occ = I->socc.as<uint8_t>();
  float* sw = I->ssw.as<float>();
  // the fused PT frame: three launches -- the queue heads and the shadow
  // count cleared, the fused launch, the film writing the totals (no
  // counters pass, no copies)
  const bool fused = n && fused_pt_shading(c, P);
  if (!fused) HIPCHK(c, hipMemsetAsync(I->dstats.p, 0, 4 * 8, s));
  if (fused) {
    const spray_rt_light& lt = P->lights[0];
    const float shade10[10] = {lt.pos[0],      lt.pos[1],      lt.pos[2], lt.radiance[0],
                               lt.radiance[1], lt.radiance[2], P->ks[0],  P->ks[1],
                               P->ks[2],       P->shininess};
    uint32_t* nshadow = I->dnum.as<uint32_t>();
    uint32_t* heads1 = c->d_heads + kHeadsBytes / sizeof(uint32_t);
    const ClearSeg cs[2] = {{heads1, kHeadsBytes, 0}, {nshadow, 4, 0}};
    HIPCHK(c, launch_clear(s, cs, 2));
    // hit records only for the per-sample records (the film needs the
    // shading and occlusion alone: 48 B per ray not written)
    HIPCHK(c, launch_scene_frame_pt(s, view(c), rays, n, rec ? hits : nullptr, shade10, occ, sv,
                                    sw, nshadow, heads1));
    HIPCHK(c, launch_film_atomic(s, image, pixid, n, ns, sw, sv, occ, scale, 4, dt, nshadow, n));
    if (rec) {
      HIPCHK(c, launch_hit_flags(s, nullptr, hits, n, I->owin.as<uint8_t>()));
      HIPCHK(c, launch_record(s, I->owin.as<uint8_t>(), n, 0, ns, samid, hits, sv, occ, *rec));
    }
  } else if (n) {
    GROW(I->oray, n * 32);
    GROW(I->ow, n * 16);
    GROW(I->ovalid, n);
    spray_rt_ray* r = I->oray.as<spray_rt_ray>();
    uint8_t* valid = I->ovalid.as<uint8_t>();
    float* w = I->ow.as<float>();
    HIPCHK(c, hipMemcpyAsync(r, rays, n * 32, hipMemcpyDeviceToDevice, s));
    HIPCHK(c, launch_path_init(s, w, valid, n));
    const int user = c->coherence;
    for (int b = 0; b < P->bounces; ++b) {
      if (b == 0) {  // camera rays: coherent packets
        c->coherence = SPRAY_RT_RAYS_COHERENT;
        const hipError_t e = launch_scene_intersect(s, view(c), r, n, hits, nullptr);
        c->coherence = user;
        HIPCHK(c, e);
      } else {
        CALL(spray_rt_intersect_scene_masked(c, r, n, valid, hits));
      }
      // the samples this bounce shades (live slots that hit), before the
      // shading pass turns the slots into the next bounce's rays
      HIPCHK(c, launch_hit_flags(s, valid, hits, n, I->owin.as<uint8_t>()));
      HIPCHK(c, launch_shade(s, *P, c->d_bsdf, c->nbsdf, b, ns, r, hits, w, valid, pixid, samid,
                             n, I->sray.as<spray_rt_ray>(), sw, sv, st, 1));
      if (ns) {
        CALL(spray_rt_occluded_scene_masked(c, I->sray.as<spray_rt_ray>(), MS, sv, occ));
        HIPCHK(c, launch_film_atomic(s, image, pixid, n, ns, sw, sv, occ, scale));
      }
      if (rec)
        HIPCHK(c, launch_record(s, I->owin.as<uint8_t>(), n, b, ns, samid, hits, sv, occ, *rec));
    }
  }
  if (before_totals) CALL(before_totals());  // the image frame's row gather
  // the group's totals: radiance rays = live slots shaded, shadows, aborts
  if (!fused) HIPCHK(c, launch_totals_of_stats(s, st, dt));
  COMM(I->tr->allreduce_u64(I, dt, 3));
  unsigned long long* ht = I->h_small + 200;
  HIPCHK(c, hipMemcpyAsync(ht, dt, 3 * 8, hipMemcpyDeviceToHost, s));
  MARK(0);
  HIPCHK(c, hipStreamSynchronize(s));
  if (totals)
    for (int k = 0; k < 3; ++k) totals[k] = ht[k];
  ++I->st[5];
  if (ht[2])
    return fail(c, SPRAY_RT_ERR_UNSUPPORTED, "%llu shading cases the reference aborts on", ht[2]);
  return SPRAY_RT_OK;
}

// SPRAY_INSITU_SPLIT_KEYS=0: the replicated PT frame's 64-bit key MIN (the
// form more than 255 domains need; kept under test)
bool split_keys() {
  static const bool on = [] {
    const char* e = std::getenv("SPRAY_INSITU_SPLIT_KEYS");
    return !(e && e[0] == '0');
  }();
  return on;
}

// C' of a replicated frame: the eye rays entering the scene's bounding box
// (idx_c, ascending), one host read of |C'| (and, want_pixmax, of the
// largest pixel id of the frame: the AO frame's sample table).
int rep_cull_select(spray_rt_insitu* I, const spray_rt_ray* rays, const int32_t* pixid, size_t n,
                    bool want_pixmax, size_t* nc_out, uint32_t* pixmax_out) {
  spray_rt_ctx* c = I->ctx;
  hipStream_t s = stream_of(c);
  SceneBox box{};
  for (int k = 0; k < 3; ++k) {
    box.lo[k] = INFINITY;
    box.hi[k] = -INFINITY;
  }
  for (int d = 0; d < c->ndom; ++d)
    for (int k = 0; k < 3; ++k) {
      box.lo[k] = std::min(box.lo[k], c->h_boxes[6 * d + k]);
      box.hi[k] = std::max(box.hi[k], c->h_boxes[6 * d + 3 + k]);
    }
  GROW(I->rfc, n);
  GROW(I->ridx_c, n * 4);
  GROW(I->rnum, 4 * 4);
  size_t t1 = 0;
  HIPCHK(c, launch_select_flagged(s, nullptr, n, nullptr, nullptr, nullptr, &t1));
  GROW(I->rsel_tmp, t1);
  uint32_t* dnum = I->rnum.as<uint32_t>();
  HIPCHK(c, launch_rep_cull(s, rays, n, box, I->rfc.as<uint8_t>()));
  HIPCHK(c, launch_select_flagged(s, I->rfc.as<uint8_t>(), n, I->ridx_c.as<uint32_t>(), dnum,
                                  I->rsel_tmp.p, &t1));
  if (want_pixmax) {
    GROW(I->rbmax, (n / kBlock + 2) * 4);
    HIPCHK(c, launch_pix_max(s, pixid, n, I->rbmax.as<uint32_t>(), dnum + 2));
  }
  HIPCHK(c, hipMemcpyAsync(I->h_small, dnum, 12, hipMemcpyDeviceToHost, s));
  HIPCHK(c, hipStreamSynchronize(s));
  ++I->st[3];
  uint32_t cnt[3];
  std::memcpy(cnt, I->h_small, 12);
  *nc_out = cnt[0];
  if (pixmax_out) *pixmax_out = want_pixmax ? cnt[2] : 0;
  return SPRAY_RT_OK;
}

// The frame with replicated eye rays (spray_rt_insitu_trace_frame): see
// include/spray_rt.h.  Every rank, over C' (the eye rays that enter the
// scene's bounding box, a superset of the rays with a domain list, the same
// ascending list on every rank without a top-level walk):
//   keyed closest hit over its domains + the point-light shading of its own
//   hit (one launch, launch_scene_rep_keyed) -> MIN all-reduce of the t bits
//   -> list positions at that t (u8 MIN, on a side stream beside the next
//   step) -> the shadow ray of every hit from the minimum t, any hit over
//   its domains (launch_scene_rep_shadows, rays built in the lanes) -> the
//   winners' flags and shadow count -> SUM all-reduce of the occlusion
//   bytes + totals -> film of its winners into per-pixel-run sums -> reduce
//   to rank 0.  One host read (|C'|).  Phases: 0 cull + select, 1 film
//   slots, 2 keyed closest hit + shading, 3 list positions, 4 shadow any
//   hit, 5 winners + totals, 6 film (collectives: kCommPhase).
int trace_replicated(spray_rt_insitu* I, const spray_rt_shader* P, const spray_rt_ray* rays,
                     const int32_t* pixid, const int32_t* samid, size_t n, int spp,
                     float* image, const spray_rt_insitu_rec* rec, unsigned long long totals[3]) {
  spray_rt_ctx* c = I->ctx;
  hipStream_t s = stream_of(c);
  const double scale = 1.0 / double(spp);
  const spray_rt_light& lt = P->lights[0];
  const float shade10[10] = {lt.pos[0],      lt.pos[1],      lt.pos[2], lt.radiance[0],
                             lt.radiance[1], lt.radiance[2], P->ks[0],  P->ks[1],
                             P->ks[2],       P->shininess};
  // ---- 1. C' (one host read: |C'| sizes the all-reduces, the same on every rank)
  MARK(0);
  size_t nc = 0;
  CALL(rep_cull_select(I, rays, pixid, n, false, &nc, nullptr));
  const uint32_t* idx_c = I->ridx_c.as<uint32_t>();
  // ---- 2. the compact film's slots (runs of equal pixels along C'), their
  // count on its way to the host while the frame runs on
  MARK(1);
  GROW(I->rincl, nc * 4 + 4);
  GROW(I->rslot_c, nc * 4 + 4);
  GROW(I->rslot_pix, nc * 4 + 4);
  GROW(I->rcompact, nc * 12 + 12);
  GROW(I->rnp, 8);
  size_t tsc = 0;
  HIPCHK(c, launch_rep_slots(s, nullptr, nullptr, nc, nullptr, nullptr, &tsc, nullptr, nullptr,
                             nullptr));
  GROW(I->rscan_tmp, tsc);
  if (!I->ev_np) HIPCHK(c, hipEventCreateWithFlags(&I->ev_np, hipEventDisableTiming));
  HIPCHK(c, launch_rep_slots(s, idx_c, pixid, nc, I->rincl.as<uint32_t>(), I->rscan_tmp.p, &tsc,
                             I->rslot_c.as<int32_t>(), I->rslot_pix.as<int32_t>(),
                             I->rnp.as<uint32_t>()));
  uint32_t* h_np = reinterpret_cast<uint32_t*>(I->h_small + 250);
  HIPCHK(c, hipMemcpyAsync(h_np, I->rnp.p, 4, hipMemcpyDeviceToHost, s));
  HIPCHK(c, hipEventRecord(I->ev_np, s));
  // ---- 3. own keyed closest hits + shading of the own hits
  MARK(2);
  GROW(I->rkeys_c, nc * 8 + 8);
  GROW(I->rtk, nc * 4 + 4);
  GROW(I->rsw, nc * 16 + 16);
  GROW(I->rsvalid, nc + 1);
  if (rec) GROW(I->rhit_c, nc * 48 + 48);
  uint64_t* keys = I->rkeys_c.as<uint64_t>();
  uint32_t* tk = I->rtk.as<uint32_t>();
  // every slot of C' is written by its lane (lanes whose ray enters no
  // resident domain write a miss and no shading: rep_ray), no prefill
  const bool split = split_keys() && c->ndom <= 255;
  HIPCHK(c, launch_scene_rep_keyed(s, view(c), rays, n, idx_c, nc, shade10,
                                   rec ? I->rhit_c.as<spray_rt_hit>() : nullptr, keys, tk,
                                   I->rsw.as<float>(), I->rsvalid.as<uint8_t>()));
  uint32_t* tstar = tk;  // the winning t of every ray (the shadow rays' origin)
  // ---- 4. the group's minimum t of every ray of C' (then the list
  // position at that t) -- split while list positions fit a byte, else the
  // 64-bit keys' MIN
  uint8_t* lp = nullptr;
  uint64_t* kmin = nullptr;
  if (split) {
    if (nc) COMM(I->tr->allreduce_min_u32(I, tk, tk, nc, 0, s));
    MARK(3);
    GROW(I->rlp, nc + 1);
    lp = I->rlp.as<uint8_t>();
    HIPCHK(c, launch_rep_lp(s, keys, tk, nc, lp));
    if (nc) {
      if (!I->cs) HIPCHK(c, hipStreamCreateWithFlags(&I->cs, hipStreamNonBlocking));
      if (!I->ev_lp0) HIPCHK(c, hipEventCreateWithFlags(&I->ev_lp0, hipEventDisableTiming));
      if (!I->ev_lp1) HIPCHK(c, hipEventCreateWithFlags(&I->ev_lp1, hipEventDisableTiming));
      if (I->tr->side_stream()) {
        HIPCHK(c, hipEventRecord(I->ev_lp0, s));
        HIPCHK(c, hipStreamWaitEvent(I->cs, I->ev_lp0, 0));
        CALL(I->tr->allreduce_min_u8(I, lp, nc, 0, I->cs));
      } else {
        COMM(I->tr->allreduce_min_u8(I, lp, nc, 0, s));
      }
      HIPCHK(c, hipEventRecord(I->ev_lp1, I->cs));
    }
  } else {
    GROW(I->rkeys_n, nc * 8 + 8);  // the minimum keys (own keys stay in keys)
    kmin = I->rkeys_n.as<uint64_t>();
    HIPCHK(c, hipMemcpyAsync(kmin, keys, nc * 8, hipMemcpyDeviceToDevice, s));
    if (nc) COMM(I->tr->allreduce_min_u64(I, kmin, nc));
    MARK(3);
    HIPCHK(c, launch_tmin_from_keys(s, kmin, nc, tk));
  }
  // ---- 5. every hit's shadow ray from the minimum t, own any hit
  MARK(4);
  GROW(I->rocc, nc + 192);
  HIPCHK(c, hipMemsetAsync(I->rocc.p, 0, nc, s));
  HIPCHK(c, launch_scene_rep_shadows(s, view(c), rays, n, idx_c, nc, tstar, shade10,
                                     I->rocc.as<uint8_t>()));
  // ---- 6. the winners (after the list positions' MIN), their shadows
  // counted behind the occlusion bytes: rank 0 counts the frame's radiance
  // rays, every rank its winners' shadow rays
  MARK(5);
  GROW(I->rwin, nc + 1);
  GROW(I->rsflag, nc + 1);  // svw: the winners' spawned shadows
  GROW(I->rnsh, kWinCounterBytes);
  HIPCHK(c, hipMemsetAsync(I->rnsh.p, 0, kWinCounterBytes, s));
  if (split && nc) HIPCHK(c, hipStreamWaitEvent(s, I->ev_lp1, 0));
  HIPCHK(c, launch_rep_win(s, keys, tk, lp, kmin, I->rsvalid.as<uint8_t>(), nc,
                           I->rwin.as<uint8_t>(), I->rsflag.as<uint8_t>(),
                           I->rnsh.as<unsigned long long>()));
  HIPCHK(c, launch_rep_totals(s, I->rocc.as<uint8_t>() + nc, I->rank == 0 ? n : 0,
                              I->rnsh.as<unsigned long long>()));
  // ---- 7. occlusion OR (a byte SUM) + totals
  COMM(I->tr->allreduce_sum_u8(I, I->rocc.as<uint8_t>(), nc + 192));
  // ---- 8. film of the rays this rank won into the runs' sums, reduced to
  // rank 0 (12 B per run of C' instead of the 16-B-per-pixel image)
  MARK(6);
  HIPCHK(c, hipEventSynchronize(I->ev_np));  // long done: the scan ran before the keyed launch
  const size_t np = nc ? *h_np : 0;
  // the all-reduces' and the reduce's payload
  const size_t pay = (split ? 5 * nc : 8 * nc) + nc + 192 + 12 * np;
  I->st[0] += pay;
  I->st[1] += pay;
  if (np) {
    HIPCHK(c, hipMemsetAsync(I->rcompact.p, 0, np * 12, s));
    HIPCHK(c, launch_film_atomic(s, I->rcompact.as<float>(), I->rslot_c.as<int32_t>(), nc, 1,
                                 I->rsw.as<float>(), I->rsflag.as<uint8_t>(),
                                 I->rocc.as<uint8_t>(), scale, 3));
    COMM(I->tr->reduce_f32(I, I->rcompact.as<float>(), np * 3, 0));
    if (I->rank == 0)
      HIPCHK(c, launch_rep_expand(s, image, I->rslot_pix.as<int32_t>(), I->rcompact.as<float>(),
                                  np));
  }
  if (rec) {
    GROW(I->rsam, nc * 4 + 4);
    HIPCHK(c, launch_gather_i32(s, idx_c, nc, samid, I->rsam.as<int32_t>()));
    HIPCHK(c, launch_record(s, I->rwin.as<uint8_t>(), nc, 0, 1, I->rsam.as<int32_t>(),
                            I->rhit_c.as<spray_rt_hit>(), I->rsflag.as<uint8_t>(),
                            I->rocc.as<uint8_t>(), *rec));
  }
  uint8_t* ht = reinterpret_cast<uint8_t*>(I->h_small + 128);  // 192 bytes
  HIPCHK(c, hipMemcpyAsync(ht, I->rocc.as<uint8_t>() + nc, 192, hipMemcpyDeviceToHost, s));
  MARK(6);
  HIPCHK(c, hipStreamSynchronize(s));
  flush_phases(I, 7);
  unsigned long long tot[3] = {0, 0, 0};
  for (int k = 0; k < 192; ++k) tot[k >> 6] += (unsigned long long)ht[k] << (k & 63);
  if (totals)
    for (int k = 0; k < 3; ++k) totals[k] = tot[k];
  ++I->st[5];
  return SPRAY_RT_OK;
}

// The replicated-ray AO frame (ooc::ShaderAo, one bounce, diffuse
// surfaces): C' and the keyed closest hit as trace_replicated, then the
// 64-bit key MIN; the winners publish their hits' shading normal and colour
// (a SUM all-reduce, 16 B per ray of C'), so every rank holds every hit's AO
// spawn input and spawns the same (source, sample) pairs
// (launch_spawn_ao_pairs, ao_ok exact); each compacts the pairs entering its
// domain boxes (launch_ao_own_flags + select) and any-hits them over its own
// domains; a SUM all-reduce of per-sample occlusion count fields (fb bits
// each, position j * ns + l) ORs the group's results; rank 0 then holds
// every weight and occlusion and films the whole frame (the other ranks'
// images stay untouched: no composite is needed).  Records: each rank its
// winners.  Totals: radiance rays n, AO rays = the pairs (the same count on
// every rank), no all-reduce.  Phases: 0 cull + select, 2 keyed closest hit,
// 3 publish, 4 AO spawn, 5 own pairs + any hit + count fields, 6 film.
// C (idx_c != null, nc rays, the largest pixel id pixmax_c): the camera
// frame's U slots, whose rays / pixels / samples the caller generated (C =
// all of them); else C' of the given eye rays.
int trace_replicated_ao(spray_rt_insitu* I, const spray_rt_shader* P, const spray_rt_ray* rays,
                        const int32_t* pixid, const int32_t* samid, size_t n, int spp,
                        float* image, const spray_rt_insitu_rec* rec,
                        unsigned long long totals[3], const uint32_t* idx_c = nullptr,
                        size_t nc_c = 0, uint32_t pixmax_c = 0, const CamFrame* cam = nullptr,
                        const CamTable* te = nullptr) {
  spray_rt_ctx* c = I->ctx;
  hipStream_t s = stream_of(c);
  const int ns = P->samples;
  size_t nc = nc_c;
  uint32_t pixmax = pixmax_c;
  MARK(0);
  if (!idx_c) {
    CALL(rep_cull_select(I, rays, pixid, n, true, &nc, &pixmax));
    idx_c = I->ridx_c.as<uint32_t>();
  }
  if (nc >= (size_t(1) << 27)) return fail(c, SPRAY_RT_ERR_LIMIT, "replicated AO: |C'| >= 2^27");
  I->last_nc_ao = nc;
  // own keyed closest hits over C' (keys and hit records at C' positions)
  MARK(2);
  GROW(I->rkeys_n, nc * 8 + 8);
  GROW(I->rhits_n, nc * 48 + 48);
  GROW(I->rkeys_c, nc * 8 + 8);
  GROW(I->rtk, nc * 4 + 4);
  const float zero10[10] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  if (cam) {
    // camera frames (C = U): only the rank's eye table E is traced, its rays
    // generated in the lanes; every other slot keeps the miss key
    HIPCHK(c, launch_fill_u64(s, I->rkeys_n.as<uint64_t>(), nc, kInsituMissKey));
    HIPCHK(c, launch_scene_cam_keyed(s, view(c), *cam, *te, zero10,
                                     I->rhits_n.as<spray_rt_hit>(), I->rkeys_n.as<uint64_t>(),
                                     I->rtk.as<uint32_t>(), nullptr, nullptr, false));
  } else {
    HIPCHK(c, launch_scene_rep_keyed(s, view(c), rays, n, idx_c, nc, zero10,
                                     I->rhits_n.as<spray_rt_hit>(), I->rkeys_n.as<uint64_t>(),
                                     I->rtk.as<uint32_t>(), nullptr, nullptr));
  }
  HIPCHK(c, hipMemcpyAsync(I->rkeys_c.p, I->rkeys_n.p, nc * 8, hipMemcpyDeviceToDevice, s));
  MARK(3);
  if (nc) COMM(I->tr->allreduce_min_u64(I, I->rkeys_c.as<uint64_t>(), nc));
  const int fb = I->world <= 3 ? 2 : (I->world <= 15 ? 4 : 8);
  const size_t npair = nc * size_t(ns);
  const size_t words = (npair * size_t(fb) + 31) / 32;
  const size_t npix = size_t(pixmax) + 1;
  GROW(I->apub, nc * 16 + 16);
  GROW(I->rwin, nc + 1);
  GROW(I->arays, nc * 32 + 32);
  GROW(I->rpix, nc * 4 + 4);
  GROW(I->rsam, nc * 4 + 4);
  GROW(I->ahits, nc * 48 + 48);
  GROW(I->apairs, npair * 4 + 4);
  GROW(I->aocc_p, npair + 1);
  GROW(I->alv, npix * size_t(ns) * 16);
  GROW(I->arec, nc * 64 + 64);
  GROW(I->ascratch, ao_scratch_bytes(nc, ns));
  GROW(I->afields, words * 4 + 4);
  GROW(I->acount, 16);
  if (rec) GROW(I->rhit_c, nc * 48 + 48);
  if (cam) GROW(I->ccomp, nc / size_t(spp) * 12 + 12);
  {  // the frame's counters, count fields, occlusion bytes and film sums in one launch
    ClearSeg cs[kClearSegs];
    int q = 0;
    cs[q++] = {I->acount.p, 16, 0};
    cs[q++] = {I->afields.p, words * 4, 0};
    cs[q++] = {I->aocc_p.p, npair, 0};
    if (cam) cs[q++] = {I->ccomp.p, nc / size_t(spp) * 12, 0};
    HIPCHK(c, launch_clear(s, cs, q));
  }
  RepAoArgs A{};
  A.nc = nc;
  A.rank = I->rank;
  A.ns = ns;
  A.fb = fb;
  A.idx_c = idx_c;
  A.keys_c = I->rkeys_c.as<uint64_t>();
  A.keys_n = I->rkeys_n.as<uint64_t>();
  A.rays = reinterpret_cast<const float4*>(rays);
  A.hits_n = I->rhits_n.as<spray_rt_hit>();
  A.pix = pixid;
  A.sam = samid;
  A.pub = I->apub.as<uint4>();
  A.win = I->rwin.as<uint8_t>();
  A.rays_c = I->arays.as<float4>();
  A.pix_c = I->rpix.as<int32_t>();
  A.sam_c = I->rsam.as<int32_t>();
  A.hit_c = rec ? I->rhit_c.as<spray_rt_hit>() : nullptr;
  A.hits_all = I->ahits.as<spray_rt_hit>();
  A.rec_ao = I->arec.as<float4>();
  A.lv = I->alv.as<float4>();
  A.fields = I->afields.as<uint32_t>();
  uint32_t* dcount = I->acount.as<uint32_t>();
  HIPCHK(c, launch_rep_ao_publish(s, A));
  // ---- 4. the winners' normals and colours on every rank
  I->st[0] += 24 * nc + 4 * words;  // the three all-reduces' payload
  I->st[1] += 24 * nc + 4 * words;
  if (nc) COMM(I->tr->allreduce_u64(I, reinterpret_cast<unsigned long long*>(A.pub), 2 * nc));
  // ---- 5. every hit's AO rays (the same pairs on every rank), own any hit
  MARK(4);
  HIPCHK(c, launch_rep_ao_hits(s, A));
  if (nc) {
    HIPCHK(c, launch_spawn_ao_pairs(s, reinterpret_cast<const spray_rt_ray*>(A.rays_c), A.hits_all,
                                    A.pix_c, nc, ns, npix, I->apairs.as<uint32_t>(),
                                    I->alv.as<float>(), I->arec.as<float>(), dcount,
                                    I->ascratch.p));
    MARK(5);
    // the pairs entering this rank's boxes, compacted and traced (the rest
    // stay 0), in two rounds: first the pairs starting in one of its
    // domains (an AO ray is mostly occluded near its start), then -- once
    // the group knows which pairs the first round occluded -- the other
    // pairs entering its boxes that are still open.  A pair occluded by its
    // home rank is not walked by the ranks its ray passes through.
    GROW(I->aflag, npair + 1);
    GROW(I->aown, npair * 4 + 4);
    const size_t nbits = (npair + 31) / 32;
    I->last_npair_ao = npair;
    GROW(I->abits, nbits * 4 + 4);
    size_t tsel = 0;
    HIPCHK(c, launch_select_flagged(s, nullptr, npair, nullptr, nullptr, nullptr, &tsel));
    GROW(I->asel_tmp, tsel);
    const uint64_t* kmin = I->rkeys_c.as<uint64_t>();
    for (int round = 1; round <= 2; ++round) {
      HIPCHK(c, launch_ao_own_flags(s, view(c), npair, I->apairs.as<uint32_t>(),
                                    I->arec.as<float>(), I->alv.as<float>(), ns, dcount,
                                    I->aflag.as<uint8_t>(), kmin, I->abits.as<uint32_t>(),
                                    round));
      HIPCHK(c, launch_select_flagged(s, I->aflag.as<uint8_t>(), npair, I->aown.as<uint32_t>(),
                                      dcount + round, I->asel_tmp.p, &tsel));
      HIPCHK(c, launch_occluded_ao_pairs(s, view(c), npair, I->apairs.as<uint32_t>(),
                                         I->arec.as<float>(), I->alv.as<float>(), ns,
                                         dcount + round, I->aocc_p.as<uint8_t>(), nullptr,
                                         I->aown.as<uint32_t>(), I->afields.as<uint32_t>(), fb));
      if (round == 1) {
        // the first round's occlusion over the group: one bit per pair, set
        // only by the pair's home rank, so a SUM of the bytes is their OR
        HIPCHK(c, launch_pack_bits(s, I->aocc_p.as<uint8_t>(), npair, I->abits.as<uint32_t>()));
        I->st[0] += 4 * nbits;
        I->st[1] += 4 * nbits;
        COMM(I->tr->allreduce_sum_u8(I, I->abits.as<uint8_t>(), nbits * 4));
      }
    }
  }
  // ---- 6. occlusion OR over the group: a SUM of the count fields' bytes
  if (words) COMM(I->tr->allreduce_sum_u8(I, I->afields.as<uint8_t>(), words * 4));
  // ---- 7. the whole film on rank 0; records of each rank's winners
  MARK(6);
  if (cam) {
    // camera frames: each rank films a slice of U's pixels, the compact
    // per-pixel sums are reduced to rank 0, which adds them to its image
    const size_t npu = nc / size_t(spp);
    const size_t q0 = npu * size_t(I->rank) / size_t(I->world);
    const size_t q1 = npu * size_t(I->rank + 1) / size_t(I->world);
    HIPCHK(c, launch_rep_ao_film_pix(s, A, spp, q0, q1, I->ccomp.as<float>(), 1.0 / double(spp)));
    if (npu) COMM(I->tr->reduce_f32(I, I->ccomp.as<float>(), npu * 3, 0));
    if (I->rank == 0 && npu)
      HIPCHK(c, launch_cam_expand(s, I->tu, cam->image_w, I->ccomp.as<float>(), image));
  } else if (I->rank == 0) {
    HIPCHK(c, launch_rep_ao_film(s, A, image, 1.0 / double(spp)));
  }
  if (rec) HIPCHK(c, launch_rep_ao_record(s, A, *rec));
  uint32_t* hp = reinterpret_cast<uint32_t*>(I->h_small + 128);
  HIPCHK(c, hipMemcpyAsync(hp, dcount, 4, hipMemcpyDeviceToHost, s));
  MARK(6);
  HIPCHK(c, hipStreamSynchronize(s));
  flush_phases(I, 7);
  if (totals) {
    totals[0] = n;
    totals[1] = *hp;
    totals[2] = 0;
  }
  ++I->st[5];
  return SPRAY_RT_OK;
}

// ---- replicated frames from the camera (spray_rt_insitu_trace_camera) ----
// The run tables of camera F (footprint.h): U, this rank's eye table E (its
// resident boxes' footprints) and shadow table S (the hit points whose
// point-light shadow ray may cross a resident box; light == null: none),
// rebuilt when the camera, the light or the residency changes.
int upload_table(spray_rt_insitu* I, const fp::Table& t, DBuf& runs, DBuf& first, CamTable* out) {
  spray_rt_ctx* c = I->ctx;
  // the previous frame's launches may still read the old table (the copies
  // below are synchronous on the null stream, not ordered after them)
  HIPCHK(c, hipStreamSynchronize(stream_of(c)));
  GROW(runs, t.runs.size() * sizeof(CamRun));
  GROW(first, t.first.size() * sizeof(uint32_t));
  HIPCHK(c, hipMemcpy(runs.p, t.runs.data(), t.runs.size() * sizeof(CamRun),
                      hipMemcpyHostToDevice));
  HIPCHK(c, hipMemcpy(first.p, t.first.data(), t.first.size() * sizeof(uint32_t),
                      hipMemcpyHostToDevice));
  out->runs = runs.as<CamRun>();
  out->first = first.as<uint32_t>();
  out->nruns = uint32_t(t.runs.size() - 1);
  out->npix = t.npix;
  return SPRAY_RT_OK;
}

int prepare_camera(spray_rt_insitu* I, const CamFrame& F, int image_h, const float* light) {
  spray_rt_ctx* c = I->ctx;
  const int n = c->ndom;
  std::vector<float> key(F.cam, F.cam + 14);
  key.push_back(float(F.image_w));
  key.push_back(float(image_h));
  for (int k = 0; k < 3; ++k) key.push_back(light ? light[k] : NAN);
  for (int d = 0; d < n; ++d)
    key.push_back(size_t(d) < c->dom2slot.size() && c->dom2slot[size_t(d)] >= 0 ? 1.f : 0.f);
  for (int k = 0; k < 6 * n; ++k) key.push_back(c->h_boxes[size_t(k)]);
  if (key.size() == I->cam_key.size() &&
      std::memcmp(key.data(), I->cam_key.data(), key.size() * sizeof(float)) == 0)
    return SPRAY_RT_OK;
  fp::Proj pj;
  if (!fp::make_proj(F.cam, &pj)) return fail(c, SPRAY_RT_ERR_ARG, "degenerate camera");
  float scene[6] = {INFINITY, INFINITY, INFINITY, -INFINITY, -INFINITY, -INFINITY};
  for (int d = 0; d < n; ++d)
    for (int k = 0; k < 3; ++k) {
      scene[k] = std::min(scene[k], c->h_boxes[6 * size_t(d) + k]);
      scene[3 + k] = std::max(scene[3 + k], c->h_boxes[6 * size_t(d) + 3 + k]);
    }
  const size_t rows = static_cast<size_t>(image_h);
  fp::Rows U(rows), E(rows), S(rows);
  bool u_all = false, e_all = false, s_all = false;
  float reg[6 * fp::kShadowSlices];
  for (int d = 0; d < n; ++d) {
    const float* b = &c->h_boxes[6 * size_t(d)];
    const bool own = size_t(d) < c->dom2slot.size() && c->dom2slot[size_t(d)] >= 0;
    const int k = fp::box_rows(pj, b, F.image_w, image_h, U);
    u_all = u_all || k == 2;
    if (!own) continue;
    e_all = e_all || fp::box_rows(pj, b, F.image_w, image_h, E) == 2;
    if (light) {
      const int ns = fp::shadow_boxes(b, scene, light, fp::kShadowSlices, reg);
      if (ns < 0) s_all = true;
      for (int q = 0; q < ns; ++q)
        s_all = s_all || fp::box_rows(pj, reg + 6 * q, F.image_w, image_h, S) == 2;
    }
  }
  const auto whole = [&](fp::Rows& r) {
    for (auto& row : r) row.assign(1, {0, F.image_w - 1});
  };
  if (u_all) whole(U);
  if (e_all) whole(E);
  fp::merge_rows(U);
  fp::merge_rows(E);
  fp::merge_rows(S);
  try {
    const fp::Table tu = fp::make_table(U, F.image_w, nullptr);
    const fp::Table te = fp::make_table(E, F.image_w, &tu);
    const fp::Table ts = fp::make_table(s_all ? U : fp::intersect_rows(S, U), F.image_w, &tu);
    if (size_t(tu.npix) * size_t(F.spp) >= (size_t(1) << 31))
      return fail(c, SPRAY_RT_ERR_LIMIT, "camera frame: |U| x spp >= 2^31");
    CALL(upload_table(I, tu, I->tu_runs, I->tu_first, &I->tu));
    CALL(upload_table(I, te, I->te_runs, I->te_first, &I->te));
    CALL(upload_table(I, ts, I->ts_runs, I->ts_first, &I->ts));
    I->tu_pixmax = tu.ymax_pix;
  } catch (const std::exception& e) {
    return fail(c, SPRAY_RT_ERR_STATE, "camera frame tables: %s", e.what());
  }
  I->cam_key.swap(key);
  return SPRAY_RT_OK;
}

// The replicated PT frame from the camera: trace_replicated's steps with U
// for C' and every device pass over this rank's own tables -- the keyed
// closest hit + shading over E's eye rays (generated in the lanes), the
// list positions, winners and film over E, the shadow any hit over S -- so
// a rank's device work follows its domains' footprints, not the frame.  No
// host read; collectives: t-bits MIN (own t bits -> group minimum), list
// positions MIN (side stream), occlusion bytes + totals SUM, the per-U-pixel
// film reduced to rank 0.  Phases as trace_replicated (0: the tables and
// prefills).
int trace_camera_pt(spray_rt_insitu* I, const spray_rt_shader* P, const CamFrame& F, int image_h,
                    float* image, const spray_rt_insitu_rec* rec, unsigned long long totals[3]) {
  spray_rt_ctx* c = I->ctx;
  hipStream_t s = stream_of(c);
  const int spp = F.spp;
  const double scale = 1.0 / double(spp);
  const spray_rt_light& lt = P->lights[0];
  const float shade10[10] = {lt.pos[0],      lt.pos[1],      lt.pos[2], lt.radiance[0],
                             lt.radiance[1], lt.radiance[2], P->ks[0],  P->ks[1],
                             P->ks[2],       P->shininess};
  MARK(0);
  CALL(prepare_camera(I, F, image_h, lt.pos));
  const size_t nu = size_t(I->tu.npix) * size_t(spp);  // U slots
  const size_t npu = I->tu.npix;                       // U pixels
  const bool split = split_keys() && c->ndom <= 255;
  I->last_nu = nu;
  GROW(I->rkeys_c, nu * 8 + 8);
  GROW(I->rtk, nu * 4 + 4);
  GROW(I->ctmin, nu * 4 + 4);
  GROW(I->rsw, nu * 16 + 16);
  GROW(I->rsvalid, nu + 1);
  GROW(I->rlp, nu + 1);
  GROW(I->rocc, nu + 192);
  GROW(I->rwin, nu + 1);
  GROW(I->rsflag, nu + 1);
  GROW(I->rnsh, kWinCounterBytes);
  GROW(I->ccomp, npu * 12 + 12);
  if (rec) GROW(I->rhit_c, nu * 48 + 48);
  uint64_t* keys = I->rkeys_c.as<uint64_t>();
  uint32_t* tk = I->rtk.as<uint32_t>();      // own t bits (0xFFFFFFFF: no own hit)
  uint32_t* tmin = I->ctmin.as<uint32_t>();  // the group's minimum
  // the frame's buffers cleared in one launch (t bits, list positions,
  // occlusion, shadow counters, film sums, winners, the keyed launch's queue
  // heads): the per-buffer memsets cost ~4 us each at N = 8
  uint32_t* heads1 = c->d_heads + kHeadsBytes / sizeof(uint32_t);
  {
    ClearSeg cs[kClearSegs];
    int ns = 0;
    cs[ns++] = {tk, nu * 4, 0xFF};
    if (split) cs[ns++] = {I->rlp.p, nu, 0xFF};
    cs[ns++] = {I->rocc.p, nu, 0};
    cs[ns++] = {I->rnsh.p, kWinCounterBytes, 0};
    cs[ns++] = {I->ccomp.p, npu * 12, 0};
    cs[ns++] = {heads1, kHeadsBytes, 0};
    if (rec) cs[ns++] = {I->rwin.p, nu, 0};
    HIPCHK(c, launch_clear(s, cs, ns));
  }
  if (!split) HIPCHK(c, launch_fill_u64(s, keys, nu, kInsituMissKey));
  // a rank with few domains tests their boxes in the lanes instead of the
  // top-level walk (the list positions then computed for its winners only)
  int nres = 0;
  for (int v : c->dom2slot) nres += v >= 0 ? 1 : 0;
  const bool direct = nres <= kDirectRes;
  const bool defer = split && direct;
  // ---- own keyed closest hits + shading over E (results at U slots)
  MARK(2);
  HIPCHK(c, launch_scene_cam_keyed(s, view(c), F, I->te, shade10,
                                   rec ? I->rhit_c.as<spray_rt_hit>() : nullptr, keys, tk,
                                   I->rsw.as<float>(), I->rsvalid.as<uint8_t>(), defer, heads1));
  // ---- the group's minimum t of every U slot (then the list position)
  uint8_t* lp = nullptr;
  uint64_t* kmin = nullptr;
  if (split) {
    if (nu) COMM(I->tr->allreduce_min_u32(I, tk, tmin, nu, 0, s));
    MARK(3);
    lp = I->rlp.as<uint8_t>();
    HIPCHK(c, launch_cam_lp(s, I->te, spp, keys, tk, tmin, lp, defer ? &F : nullptr,
                            c->d_boxes, c->d_tlas, c->ntlas));
    if (nu) {
      if (!I->cs) HIPCHK(c, hipStreamCreateWithFlags(&I->cs, hipStreamNonBlocking));
      if (!I->ev_lp0) HIPCHK(c, hipEventCreateWithFlags(&I->ev_lp0, hipEventDisableTiming));
      if (!I->ev_lp1) HIPCHK(c, hipEventCreateWithFlags(&I->ev_lp1, hipEventDisableTiming));
      if (I->tr->side_stream()) {
        HIPCHK(c, hipEventRecord(I->ev_lp0, s));
        HIPCHK(c, hipStreamWaitEvent(I->cs, I->ev_lp0, 0));
        CALL(I->tr->allreduce_min_u8(I, lp, nu, 0, I->cs));
      } else {
        COMM(I->tr->allreduce_min_u8(I, lp, nu, 0, s));
      }
      HIPCHK(c, hipEventRecord(I->ev_lp1, I->cs));
    }
  } else {
    GROW(I->rkeys_n, nu * 8 + 8);
    kmin = I->rkeys_n.as<uint64_t>();
    HIPCHK(c, hipMemcpyAsync(kmin, keys, nu * 8, hipMemcpyDeviceToDevice, s));
    if (nu) COMM(I->tr->allreduce_min_u64(I, kmin, nu));
    MARK(3);
    HIPCHK(c, launch_tmin_from_keys(s, kmin, nu, tmin));
  }
  // ---- the shadow ray of every hit in S from the minimum t, own any hit
  MARK(4);
  HIPCHK(c, launch_scene_cam_shadows(s, view(c), F, I->ts, tmin, shade10, I->rocc.as<uint8_t>(),
                                     direct));
  // ---- the winners among E's slots, their shadows counted
  MARK(5);
  if (split && nu) HIPCHK(c, hipStreamWaitEvent(s, I->ev_lp1, 0));
  HIPCHK(c, launch_cam_win(s, I->te, spp, keys, tk, tmin, lp, kmin, I->rsvalid.as<uint8_t>(),
                           I->rwin.as<uint8_t>(), I->rsflag.as<uint8_t>(),
                           I->rnsh.as<unsigned long long>()));
  const unsigned long long nrad = I->rank == 0 ? (unsigned long long)F.image_w *
                                                     (unsigned long long)image_h *
                                                     (unsigned long long)spp
                                               : 0ull;
  HIPCHK(c, launch_rep_totals(s, I->rocc.as<uint8_t>() + nu, nrad,
                              I->rnsh.as<unsigned long long>()));
  // ---- occlusion OR (a byte SUM) + totals
  COMM(I->tr->allreduce_sum_u8(I, I->rocc.as<uint8_t>(), nu + 192));
  // ---- film of the rank's winners into per-U-pixel sums, reduced to rank 0
  MARK(6);
  const size_t pay = (split ? 5 * nu : 8 * nu) + nu + 192 + 12 * npu;
  I->st[0] += pay;
  I->st[1] += pay;
  if (npu) {
    HIPCHK(c, launch_cam_film(s, I->te, spp, I->ccomp.as<float>(), I->rsw.as<float>(),
                              I->rsflag.as<uint8_t>(), I->rocc.as<uint8_t>(), scale));
    COMM(I->tr->reduce_f32(I, I->ccomp.as<float>(), npu * 3, 0));
    if (I->rank == 0)
      HIPCHK(c, launch_cam_expand(s, I->tu, F.image_w, I->ccomp.as<float>(), image));
  }
  if (rec)
    HIPCHK(c, launch_cam_record(s, I->te, spp, F.image_w, I->rwin.as<uint8_t>(),
                                I->rhit_c.as<spray_rt_hit>(), I->rsflag.as<uint8_t>(),
                                I->rocc.as<uint8_t>(), *rec));
  uint8_t* ht = reinterpret_cast<uint8_t*>(I->h_small + 128);  // 192 bytes
  HIPCHK(c, hipMemcpyAsync(ht, I->rocc.as<uint8_t>() + nu, 192, hipMemcpyDeviceToHost, s));
  MARK(6);
  HIPCHK(c, hipStreamSynchronize(s));
  flush_phases(I, 7);
  unsigned long long tot[3] = {0, 0, 0};
  for (int k = 0; k < 192; ++k) tot[k >> 6] += (unsigned long long)ht[k] << (k & 63);
  if (totals)
    for (int k = 0; k < 3; ++k) totals[k] = tot[k];
  ++I->st[5];
  return SPRAY_RT_OK;
}

// The replicated AO frame from the camera: U's eye rays, pixels and samples
// generated into U-ordered arrays (one pass; the spawn and film read them),
// then trace_replicated_ao over C = U with the keyed closest hit over the
// rank's eye table E only (its rays generated in the lanes).
int trace_camera_ao(spray_rt_insitu* I, const spray_rt_shader* P, const CamFrame& F, int image_h,
                    float* image, const spray_rt_insitu_rec* rec, unsigned long long totals[3]) {
  spray_rt_ctx* c = I->ctx;
  hipStream_t s = stream_of(c);
  MARK(0);
  CALL(prepare_camera(I, F, image_h, nullptr));
  const size_t nu = size_t(I->tu.npix) * size_t(F.spp);
  GROW(I->crays, nu * 32 + 32);
  GROW(I->cpix, nu * 4 + 4);
  GROW(I->csam, nu * 4 + 4);
  if (I->ciota_n < nu) {
    GROW(I->ciota, nu * 4 + 4);
    HIPCHK(c, launch_iota_u32(s, I->ciota.as<uint32_t>(), nu));
    I->ciota_n = nu;
  }
  HIPCHK(c, launch_cam_eye_rays(s, I->tu, F, I->crays.as<spray_rt_ray>(), I->cpix.as<int32_t>(),
                                I->csam.as<int32_t>()));
  const size_t n = size_t(F.image_w) * size_t(image_h) * size_t(F.spp);
  return trace_replicated_ao(I, P, I->crays.as<spray_rt_ray>(), I->cpix.as<int32_t>(),
                             I->csam.as<int32_t>(), n, F.spp, image, rec, totals,
                             I->ciota.as<uint32_t>(), nu, I->tu_pixmax, &F, &I->te);
}

void free_all(spray_rt_insitu* I) {
  DBuf* all[] = {&I->hray[0], &I->hray[1], &I->hw[0], &I->hw[1], &I->hpix[0], &I->hpix[1],
                 &I->hsam[0], &I->hsam[1], &I->mask, &I->idx, &I->starts, &I->plan_tmp,
                 &I->dcnt, &I->sendb, &I->recvb, &I->oray, &I->ow, &I->opix, &I->osam,
                 &I->ohit, &I->okey, &I->obest, &I->owin, &I->ovalid, &I->best, &I->keyback,
                 &I->sray, &I->ssw, &I->ssv, &I->socc, &I->ssel, &I->smask,
                 &I->sidx, &I->sstarts, &I->ashadow, &I->aocc, &I->sret, &I->nsel,
                 &I->sel_tmp, &I->dnum, &I->dstats, &I->dtot, &I->rfc,
                 &I->ridx_c, &I->rnum, &I->rsel_tmp, &I->rkeys_n, &I->rhits_n,
                 &I->rkeys_c, &I->rsray, &I->rsflag, &I->rwin, &I->rsvalid, &I->rsw, &I->rocc,
                 &I->rpix, &I->rsam, &I->rhit_c, &I->rnsh, &I->apub, &I->arays,
                 &I->ahits, &I->apairs, &I->aocc_p, &I->alv, &I->arec, &I->ascratch,
                 &I->afields, &I->acount, &I->rincl, &I->rscan_tmp,
                 &I->rslot_c, &I->rslot_pix, &I->rcompact, &I->rnp, &I->rtk, &I->rlp, &I->rbmax,
                 &I->aflag, &I->aown, &I->asel_tmp, &I->abits, &I->tu_runs, &I->tu_first,
                 &I->te_runs, &I->te_first, &I->ts_runs, &I->ts_first, &I->ctmin, &I->ccomp,
                 &I->crays, &I->cpix, &I->csam, &I->ciota, &I->gpack, &I->ti_runs,
                 &I->ti_first, &I->tg_runs, &I->tg_first};
  for (DBuf* b : all)
    if (b->p) (void)hipFree(b->p);
  for (hipEvent_t e : I->ev)
    if (e) (void)hipEventDestroy(e);
  if (I->ev_np) (void)hipEventDestroy(I->ev_np);
  if (I->ev_lp0) (void)hipEventDestroy(I->ev_lp0);
  if (I->ev_lp1) (void)hipEventDestroy(I->ev_lp1);
  if (I->cs) (void)hipStreamDestroy(I->cs);
  if (I->h_small) (void)hipHostFree(I->h_small);
}

// Morton::expandBits / compute (src/render/morton.h:32-50)
uint32_t expand_bits(uint32_t v) {
  v = (v * 0x00010001u) & 0xFF0000FFu;
  v = (v * 0x00000101u) & 0x0F00F00Fu;
  v = (v * 0x00000011u) & 0xC30C30C3u;
  v = (v * 0x00000005u) & 0x49249249u;
  return v;
}
uint32_t morton(float x, float y, float z) {
  x = std::min(std::max(x * 1024.0f, 0.0f), 1023.0f);
  y = std::min(std::max(y * 1024.0f, 0.0f), 1023.0f);
  z = std::min(std::max(z * 1024.0f, 0.0f), 1023.0f);
  return expand_bits(uint32_t(x)) * 4 + expand_bits(uint32_t(y)) * 2 + expand_bits(uint32_t(z));
}

}  // namespace

extern "C" {

int spray_rt_insitu_unique_id(void* id_out, size_t bytes) {
  if (!id_out || bytes < sizeof(ncclUniqueId)) return SPRAY_RT_ERR_ARG;
  const NcclApi& N = nccl();
  if (!N.ok) return SPRAY_RT_ERR_UNSUPPORTED;
  ncclUniqueId id;
  if (N.GetUniqueId(&id) != ncclSuccess) return SPRAY_RT_ERR_HIP;
  std::memcpy(id_out, &id, sizeof(id));
  return SPRAY_RT_OK;
}

int spray_rt_insitu_create(spray_rt_ctx_t c, int world, int rank, const void* nccl_id,
                           const spray_rt_transport* host, spray_rt_insitu_t* out) {
  if (!c || !out) return SPRAY_RT_ERR_ARG;
  *out = nullptr;
  if (world < 1 || world > 64 || rank < 0 || rank >= world)
    return fail(c, SPRAY_RT_ERR_ARG, "in-situ group: world %d rank %d (world in [1, 64])", world,
                rank);
  if (!nccl_id && !host)
    return fail(c, SPRAY_RT_ERR_ARG, "in-situ group needs an RCCL id or host collectives");
  spray_rt_transport cb{};
  if (!nccl_id) {
    // struct_size first, before any callback field is read (spray_rt.h: a
    // layout-1 caller's `user` pointer lands here and fails the range check)
    const size_t have = host->struct_size;
    if (have < offsetof(spray_rt_transport, allreduce_min_u64) ||
        have > SPRAY_RT_TRANSPORT_MAX_SIZE)
      return fail(c, SPRAY_RT_ERR_ARG,
                  "spray_rt_transport.struct_size %zu outside [%zu, %d] (layout %d expected)",
                  have, offsetof(spray_rt_transport, allreduce_min_u64),
                  SPRAY_RT_TRANSPORT_MAX_SIZE, SPRAY_RT_TRANSPORT_ABI);
    std::memcpy(&cb, host, std::min(have, sizeof(spray_rt_transport)));
    cb.struct_size = sizeof(spray_rt_transport);
    if (!cb.alltoallv || !cb.allreduce_u64 || !cb.reduce_f32)
      return fail(c, SPRAY_RT_ERR_ARG, "host collectives: alltoallv / allreduce_u64 / "
                                       "reduce_f32 are required");
  }
  HIPCHK(c, hipSetDevice(c->device));
  std::unique_ptr<spray_rt_insitu> I(new (std::nothrow) spray_rt_insitu);
  if (!I) return SPRAY_RT_ERR_NOMEM;
  I->ctx = c;
  I->world = world;
  I->rank = rank;
  HIPCHK(c, hipHostMalloc(reinterpret_cast<void**>(&I->h_small), 256 * 8, hipHostMallocDefault));
  if (nccl_id) {
    const NcclApi& N = nccl();
    if (!N.ok) {
      free_all(I.get());
      return fail(c, SPRAY_RT_ERR_UNSUPPORTED, "RCCL unavailable: %s", N.err.c_str());
    }
    auto t = std::make_unique<RcclTransport>();
    const char* self = std::getenv("SPRAY_INSITU_NCCL_SELF");
    t->self_via_nccl = self && self[0] == '1';
    ncclUniqueId id;
    std::memcpy(&id, nccl_id, sizeof(id));
    const ncclResult_t r = N.CommInitRank(&t->comm, world, id, rank);
    if (r != ncclSuccess) {
      free_all(I.get());
      return fail(c, SPRAY_RT_ERR_HIP, "ncclCommInitRank: %s", N.GetErrorString(r));
    }
    I->tr = std::move(t);
  } else {
    auto t = std::make_unique<HostTransport>();
    t->cb = cb;  // validated above; callbacks past the caller's struct_size stay NULL
    if (const char* lk = std::getenv("SPRAY_INSITU_SERIAL"))
      if (lk[0]) t->lock_fd = open(lk, O_RDWR | O_CREAT, 0666);
    I->tr = std::move(t);
  }
  *out = I.release();
  return SPRAY_RT_OK;
}

int spray_rt_insitu_create_replay(spray_rt_ctx_t c, int world, int rank,
                                  spray_rt_insitu_t* out) {
  if (!c || !out) return SPRAY_RT_ERR_ARG;
  *out = nullptr;
  if (world < 1 || world > 64 || rank < 0 || rank >= world)
    return fail(c, SPRAY_RT_ERR_ARG, "in-situ group: world %d rank %d (world in [1, 64])", world,
                rank);
  HIPCHK(c, hipSetDevice(c->device));
  std::unique_ptr<spray_rt_insitu> I(new (std::nothrow) spray_rt_insitu);
  if (!I) return SPRAY_RT_ERR_NOMEM;
  I->ctx = c;
  I->world = world;
  I->rank = rank;
  HIPCHK(c, hipHostMalloc(reinterpret_cast<void**>(&I->h_small), 256 * 8, hipHostMallocDefault));
  I->tr = std::make_unique<ReplayTransport>();
  *out = I.release();
  return SPRAY_RT_OK;
}

int spray_rt_insitu_replay_set(spray_rt_insitu_t I, const uint32_t* d_tmin,
                               const uint8_t* d_lpmin, size_t n) {
  if (!I) return SPRAY_RT_ERR_ARG;
  auto* t = dynamic_cast<ReplayTransport*>(I->tr.get());
  if (!t) return fail(I->ctx, SPRAY_RT_ERR_STATE, "not a replay context");
  if (n && (!is_device_ptr(d_tmin) || !is_device_ptr(d_lpmin)))
    return fail(I->ctx, SPRAY_RT_ERR_ARG, "replay arrays must be device memory");
  t->tmin = d_tmin;
  t->lpmin = d_lpmin;
  t->n = n;
  return SPRAY_RT_OK;
}

int spray_rt_insitu_replay_set_ao(spray_rt_insitu_t I, const uint64_t* d_kmin,
                                  const uint64_t* d_pub, size_t n) {
  if (!I) return SPRAY_RT_ERR_ARG;
  auto* t = dynamic_cast<ReplayTransport*>(I->tr.get());
  if (!t) return fail(I->ctx, SPRAY_RT_ERR_STATE, "not a replay context");
  if (n && (!is_device_ptr(d_kmin) || !is_device_ptr(d_pub)))
    return fail(I->ctx, SPRAY_RT_ERR_ARG, "replay arrays must be device memory");
  t->kmin = d_kmin;
  t->pub = d_pub;
  t->nk = n;
  return SPRAY_RT_OK;
}

int spray_rt_insitu_replay_bits_ao(spray_rt_insitu_t I, const uint8_t* d_bits, uint8_t* d_out,
                                   size_t nbytes, size_t* n) {
  if (!I || !n) return SPRAY_RT_ERR_ARG;
  auto* t = dynamic_cast<ReplayTransport*>(I->tr.get());
  if (!t) return fail(I->ctx, SPRAY_RT_ERR_STATE, "not a replay context");
  *n = I->abits.p ? (I->last_npair_ao + 31) / 32 * 4 : 0;
  if (d_out) {  // the last frame's own first-round bits
    if (nbytes < *n) return fail(I->ctx, SPRAY_RT_ERR_LIMIT, "replay bits: cap %zu < %zu",
                                 nbytes, *n);
    hipStream_t s = stream_of(I->ctx);
    HIPCHK(I->ctx, hipMemcpyAsync(d_out, I->abits.p, *n, hipMemcpyDeviceToDevice, s));
    HIPCHK(I->ctx, hipStreamSynchronize(s));
    return SPRAY_RT_OK;
  }
  if (d_bits && !is_device_ptr(d_bits))
    return fail(I->ctx, SPRAY_RT_ERR_ARG, "replay arrays must be device memory");
  t->bits = d_bits;
  t->nbits_bytes = d_bits ? nbytes : 0;
  return SPRAY_RT_OK;
}

int spray_rt_insitu_replay_capture_ao(spray_rt_insitu_t I, uint64_t* d_kmin, uint64_t* d_pub,
                                      size_t cap, size_t* n) {
  if (!I || !n) return SPRAY_RT_ERR_ARG;
  spray_rt_ctx* c = I->ctx;
  if (I->cam_key.empty() || !I->rkeys_c.p || !I->apub.p || !I->last_nc_ao)
    return fail(c, SPRAY_RT_ERR_STATE, "no replicated AO camera frame traced yet");
  const size_t m = I->last_nc_ao;
  *n = m;
  if (!d_kmin || !d_pub) return SPRAY_RT_OK;  // size query
  if (cap < m) return fail(c, SPRAY_RT_ERR_LIMIT, "replay capture: %zu slots, cap %zu", m, cap);
  hipStream_t s = stream_of(c);
  HIPCHK(c, hipMemcpyAsync(d_kmin, I->rkeys_c.p, m * 8, hipMemcpyDeviceToDevice, s));
  HIPCHK(c, hipMemcpyAsync(d_pub, I->apub.p, m * 16, hipMemcpyDeviceToDevice, s));
  HIPCHK(c, hipStreamSynchronize(s));
  return SPRAY_RT_OK;
}

int spray_rt_insitu_replay_capture(spray_rt_insitu_t I, uint32_t* d_tmin, uint8_t* d_lpmin,
                                   size_t cap, size_t* n) {
  if (!I || !n) return SPRAY_RT_ERR_ARG;
  spray_rt_ctx* c = I->ctx;
  // U slots of the last camera frame: the U pixels times its spp (the
  // group MIN arrays were sized for them)
  if (I->cam_key.empty() || !I->ctmin.p || !I->rlp.p)
    return fail(c, SPRAY_RT_ERR_STATE, "no replicated camera frame traced yet");
  const size_t m = I->last_nu;
  *n = m;
  if (!d_tmin || !d_lpmin) return SPRAY_RT_OK;  // size query
  if (cap < m) return fail(c, SPRAY_RT_ERR_LIMIT, "replay capture: %zu slots, cap %zu", m, cap);
  hipStream_t s = stream_of(c);
  HIPCHK(c, hipMemcpyAsync(d_tmin, I->ctmin.p, m * 4, hipMemcpyDeviceToDevice, s));
  HIPCHK(c, hipMemcpyAsync(d_lpmin, I->rlp.p, m, hipMemcpyDeviceToDevice, s));
  HIPCHK(c, hipStreamSynchronize(s));
  return SPRAY_RT_OK;
}

int spray_rt_insitu_destroy(spray_rt_insitu_t I) {
  if (!I) return SPRAY_RT_ERR_ARG;
  (void)hipSetDevice(I->ctx->device);
  (void)hipStreamSynchronize(stream_of(I->ctx));
  free_all(I);
  delete I;
  return SPRAY_RT_OK;
}

int spray_rt_insitu_partition(const float* boxes, int n, const float sb[6], int nranks,
                              int* owner) {
  return spray_rt_insitu_partition_mode(boxes, n, sb, nranks, SPRAY_RT_PARTITION_GROUP_CLOSE,
                                        owner);
}

int spray_rt_insitu_partition_mode(const float* boxes, int n, const float sb[6], int nranks,
                                   int mode, int* owner) {
  if (!boxes || !sb || !owner || n < 0 || nranks <= 0) return SPRAY_RT_ERR_ARG;
  if (mode != SPRAY_RT_PARTITION_GROUP_CLOSE && mode != SPRAY_RT_PARTITION_ROUND_ROBIN)
    return SPRAY_RT_ERR_ARG;
  // scale + offset of the unit-cube transform, evaluated as glm's
  // trans * scale matrix applied to (c, 1): fl(fl(s * c) + off)
  float scale[3], off[3];
  for (int j = 0; j < 3; ++j) {
    const float diag = sb[3 + j] - sb[j];
    scale[j] = 1.0f / diag;
    off[j] = 0.0f - sb[j] * scale[j];
  }
  std::vector<std::pair<uint32_t, int>> codes(n);
  for (int i = 0; i < n; ++i) {
    float cc[3];
    for (int j = 0; j < 3; ++j) {
      const float center = (boxes[6 * i + j] + boxes[6 * i + 3 + j]) * 0.5f;  // Aabb::getCenter
      cc[j] = center * scale[j] + off[j];
    }
    codes[i] = {morton(cc[0], cc[1], cc[2]), i};
  }
  // std::sort by code leaves equal codes unordered; the id makes it total
  std::sort(codes.begin(), codes.end());
  if (mode == SPRAY_RT_PARTITION_ROUND_ROBIN) {  // data_partition.h:139-155
    int rank = 0;
    for (const auto& cd : codes) {
      owner[cd.second] = rank;
      if (++rank == nranks) rank = 0;
    }
    return SPRAY_RT_OK;
  }
  const int shares = n / nranks;
  int rank = 0, s = 0;
  for (const auto& cd : codes) {
    owner[cd.second] = rank;
    if (++s == shares) {
      s = 0;
      if (++rank == nranks) rank = 0;
    }
  }
  return SPRAY_RT_OK;
}

int spray_rt_insitu_trace(spray_rt_insitu_t I, const spray_rt_shader* P, const spray_rt_ray* rays,
                          const int32_t* pixid, const int32_t* samid, size_t n, int spp,
                          float* image, const spray_rt_insitu_rec* rec,
                          unsigned long long totals[3]) {
  if (!I) return SPRAY_RT_ERR_ARG;
  spray_rt_ctx* c = I->ctx;
  if (spray_rt_shadow_slots(P) < 0 || spp <= 0)
    return fail(c, SPRAY_RT_ERR_ARG, "bad shader configuration");
  if (rec && (spray_rt_shadow_slots(P) > 64 || !rec->d_count || !is_device_ptr(rec->d_count)))
    return fail(c, SPRAY_RT_ERR_ARG, "records need <= 64 shadow slots and a device counter");
  if (n > 0xFFFFFFFFull) return fail(c, SPRAY_RT_ERR_LIMIT, "n > 2^32");
  if (!image || !is_device_ptr(image) ||
      (n && (!is_device_ptr(rays) || !is_device_ptr(pixid) || !is_device_ptr(samid))))
    return fail(c, SPRAY_RT_ERR_ARG, "in-situ trace needs device buffers");
  int r = scene_common(c, image, 1, image);
  if (r) return r;
  if (!c->d_owner) return fail(c, SPRAY_RT_ERR_STATE, "no owner map set");
  // every domain local: the frame needs no exchange (trace_local).  The full
  // protocol stays selectable (SPRAY_INSITU_LOCAL=0) and is what a test of
  // the self exchange through RCCL (SPRAY_INSITU_NCCL_SELF=1) runs.
  const char* lo = std::getenv("SPRAY_INSITU_LOCAL");
  const bool local_ok = !(lo && lo[0] == '0') && I->tr->self_direct();
  I->nev = 0;
  I->tr->serial_begin();
  if (local_ok && all_local(I)) {
    r = trace_local(I, P, rays, pixid, samid, n, spp, image, rec, totals);
    flush_phases(I, 1);
  } else {
    r = trace(I, P, rays, pixid, samid, n, spp, image, rec, totals);
  }
  I->tr->serial_end();
  return r;
}

int spray_rt_insitu_trace_frame(spray_rt_insitu_t I, const spray_rt_shader* P,
                                const spray_rt_ray* rays, const int32_t* pixid,
                                const int32_t* samid, size_t n, int spp, float* image,
                                const spray_rt_insitu_rec* rec, unsigned long long totals[3]) {
  if (!I) return SPRAY_RT_ERR_ARG;
  spray_rt_ctx* c = I->ctx;
  if (spray_rt_shadow_slots(P) < 0 || spp <= 0)
    return fail(c, SPRAY_RT_ERR_ARG, "bad shader configuration");
  if (rec && (!rec->d_count || !is_device_ptr(rec->d_count)))
    return fail(c, SPRAY_RT_ERR_ARG, "records need a device counter");
  if (n > 0xFFFFFFFFull) return fail(c, SPRAY_RT_ERR_LIMIT, "n > 2^32");
  if (!image || !is_device_ptr(image) ||
      (n && (!is_device_ptr(rays) || !is_device_ptr(pixid) || !is_device_ptr(samid))))
    return fail(c, SPRAY_RT_ERR_ARG, "in-situ trace needs device buffers");
  int r = scene_common(c, image, 1, image);
  if (r) return r;
  if (!c->d_owner) return fail(c, SPRAY_RT_ERR_STATE, "no owner map set");
  const bool ao = P->shader == SPRAY_RT_SHADER_AO && P->bounces == 1 && !c->bsdf_delta &&
                  P->samples >= 1 && P->samples <= 32;
  if (!fused_pt_shading(c, P) && !ao)
    return fail(c, SPRAY_RT_ERR_UNSUPPORTED,
                "replicated frames need one bounce, diffuse surfaces and one point light "
                "(PT) or <= 32 samples (AO)");
  if (!I->tr->has_rep())
    return fail(c, SPRAY_RT_ERR_UNSUPPORTED,
                "the host transport gives no allreduce_min_u64 / allreduce_sum_u8");
  // SPRAY_INSITU_REPLICATED=1: the replicated steps even at world 1 (their
  // collectives through a one-rank communicator: the product transport's
  // calls on a one-GPU box)
  const char* fr = std::getenv("SPRAY_INSITU_REPLICATED");
  const bool force_rep = fr && fr[0] == '1';
  I->nev = 0;
  I->tr->serial_begin();
  if (I->world == 1 && !force_rep) {
    r = trace_local(I, P, rays, pixid, samid, n, spp, image, rec, totals);
    flush_phases(I, 1);
  } else {
    r = ao ? trace_replicated_ao(I, P, rays, pixid, samid, n, spp, image, rec, totals)
           : trace_replicated(I, P, rays, pixid, samid, n, spp, image, rec, totals);
  }
  I->tr->serial_end();
  return r;
}

int spray_rt_insitu_trace_camera(spray_rt_insitu_t I, const spray_rt_shader* P,
                                 const float cam[14], int image_w, int image_h, int spp,
                                 float* image, const spray_rt_insitu_rec* rec,
                                 unsigned long long totals[3]) {
  if (!I || !cam) return SPRAY_RT_ERR_ARG;
  spray_rt_ctx* c = I->ctx;
  if (spray_rt_shadow_slots(P) < 0 || spp <= 0 || image_w <= 0 || image_h <= 0)
    return fail(c, SPRAY_RT_ERR_ARG, "bad shader or frame configuration");
  if (float(image_w) != cam[12] || float(image_h) != cam[13])
    return fail(c, SPRAY_RT_ERR_ARG, "the camera record is for a %gx%g image", cam[12], cam[13]);
  if (rec && (!rec->d_count || !is_device_ptr(rec->d_count)))
    return fail(c, SPRAY_RT_ERR_ARG, "records need a device counter");
  const size_t n = size_t(image_w) * size_t(image_h) * size_t(spp);
  if (n > 0x7FFFFFFFull) return fail(c, SPRAY_RT_ERR_LIMIT, "frame > 2^31 samples");
  if (!image || !is_device_ptr(image)) return fail(c, SPRAY_RT_ERR_ARG, "needs a device image");
  int r = scene_common(c, image, 1, image);
  if (r) return r;
  if (!c->d_owner) return fail(c, SPRAY_RT_ERR_STATE, "no owner map set");
  const bool ao = P->shader == SPRAY_RT_SHADER_AO && P->bounces == 1 && !c->bsdf_delta &&
                  P->samples >= 1 && P->samples <= 32;
  if (!fused_pt_shading(c, P) && !ao)
    return fail(c, SPRAY_RT_ERR_UNSUPPORTED,
                "replicated frames need one bounce, diffuse surfaces and one point light "
                "(PT) or <= 32 samples (AO)");
  if (!I->tr->has_rep())
    return fail(c, SPRAY_RT_ERR_UNSUPPORTED,
                "the host transport gives no allreduce_min_u64 / allreduce_sum_u8");
  CamFrame F{};
  for (int k = 0; k < 14; ++k) F.cam[k] = cam[k];
  F.image_w = image_w;
  F.spp = spp;
  const char* fr = std::getenv("SPRAY_INSITU_REPLICATED");
  const bool force_rep = fr && fr[0] == '1';
  // one rank: the one-band image frame (U's eye rays, then the all-local
  // fused frame); every domain is resident at world 1
  if (I->world == 1 && !force_rep)
    return spray_rt_insitu_trace_image(I, P, cam, image_w, image_h, spp, 1, image, rec, totals);
  I->nev = 0;
  I->tr->serial_begin();
  r = ao ? trace_camera_ao(I, P, F, image_h, image, rec, totals)
         : trace_camera_pt(I, P, F, image_h, image, rec, totals);
  I->tr->serial_end();
  return r;
}

// Rows of band b of bt bands over h rows: [b h / bt, (b + 1) h / bt).
inline int band_row(int b, int bt, int h) { return int((long long)b * h / bt); }

// The image frame's eye-ray table: U (the pixels whose eye rays may enter a
// domain box: the union of every box's screen footprint, footprint.h)
// restricted to this rank's bands, rebuilt when the camera, the boxes or the
// split change; img_upix = U's pixels over the whole image.
int prepare_image(spray_rt_insitu* I, const float cam[14], int image_w, int image_h, int bands) {
  spray_rt_ctx* c = I->ctx;
  const int n = c->ndom;
  std::vector<float> key(cam, cam + 14);
  for (int v : {image_w, image_h, bands, I->world, I->rank}) key.push_back(float(v));
  for (int k = 0; k < 6 * n; ++k) key.push_back(c->h_boxes[size_t(k)]);
  if (key.size() == I->img_key.size() &&
      std::memcmp(key.data(), I->img_key.data(), key.size() * sizeof(float)) == 0)
    return SPRAY_RT_OK;
  fp::Proj pj;
  if (!fp::make_proj(cam, &pj)) return fail(c, SPRAY_RT_ERR_ARG, "degenerate camera");
  uint64_t upix = 0;
  fp::Rows U = fp::union_rows(pj, c->h_boxes.data(), n, image_w, image_h, &upix);
  const int bt = I->world * bands;
  // rank k's pixels of U, its rows in ascending order (its table's order);
  // rank 0 also gets the other ranks' runs, rank by rank (the gather's order)
  fp::Table mine, others;
  I->img_counts.assign(size_t(I->world), 0u);
  for (int k = 0; k < I->world; ++k) {
    fp::Table& t = k == I->rank ? mine : others;
    if (k != I->rank && !(I->rank == 0 && k > 0)) {
      uint32_t n = 0;
      for (int b = k; b < bt; b += I->world)
        for (int y = band_row(b, bt, image_h); y < band_row(b + 1, bt, image_h); ++y)
          for (const auto& iv : U[size_t(y)]) n += uint32_t(iv.second - iv.first + 1);
      I->img_counts[size_t(k)] = n;
      continue;
    }
    const uint32_t np0 = t.npix;
    for (int b = k; b < bt; b += I->world)
      for (int y = band_row(b, bt, image_h); y < band_row(b + 1, bt, image_h); ++y)
        for (const auto& iv : U[size_t(y)]) {
          t.runs.push_back(CamRun{y, iv.first, t.npix, t.npix});
          t.npix += uint32_t(iv.second - iv.first + 1);
        }
    I->img_counts[size_t(k)] = t.npix - np0;
  }
  fp::finish_table(mine);
  fp::finish_table(others);
  CALL(upload_table(I, mine, I->ti_runs, I->ti_first, &I->ti));
  CALL(upload_table(I, others, I->tg_runs, I->tg_first, &I->tg));
  I->img_upix = upix;
  I->img_key.swap(key);
  return SPRAY_RT_OK;
}

int spray_rt_insitu_trace_image(spray_rt_insitu_t I, const spray_rt_shader* P,
                                const float cam[14], int image_w, int image_h, int spp, int bands,
                                float* image, const spray_rt_insitu_rec* rec,
                                unsigned long long totals[3]) {
  if (!I || !cam) return SPRAY_RT_ERR_ARG;
  spray_rt_ctx* c = I->ctx;
  if (spray_rt_shadow_slots(P) < 0 || spp <= 0 || image_w <= 0 || image_h <= 0 || bands <= 0)
    return fail(c, SPRAY_RT_ERR_ARG, "bad shader or frame configuration");
  if (float(image_w) != cam[12] || float(image_h) != cam[13])
    return fail(c, SPRAY_RT_ERR_ARG, "the camera record is for a %gx%g image", cam[12], cam[13]);
  const int W = I->world, bt = W * bands;
  if (bt > image_h) return fail(c, SPRAY_RT_ERR_ARG, "%d bands over %d rows", bt, image_h);
  if (rec && (spray_rt_shadow_slots(P) > 64 || !rec->d_count || !is_device_ptr(rec->d_count)))
    return fail(c, SPRAY_RT_ERR_ARG, "records need <= 64 shadow slots and a device counter");
  if (size_t(image_w) * size_t(image_h) * size_t(spp) > 0x7FFFFFFFull)
    return fail(c, SPRAY_RT_ERR_LIMIT, "frame > 2^31 samples");
  if (!image || !is_device_ptr(image)) return fail(c, SPRAY_RT_ERR_ARG, "needs a device image");
  int r = scene_common(c, image, 1, image);
  if (r) return r;
  // image-parallel: every domain resident on every rank (the reference's ooc
  // mode, where any rank may load any domain)
  for (int d = 0; d < c->ndom; ++d)
    if (size_t(d) >= c->dom2slot.size() || c->dom2slot[size_t(d)] < 0)
      return fail(c, SPRAY_RT_ERR_STATE,
                  "image-parallel frames need every domain resident (domain %d is not)", d);
  hipStream_t s = stream_of(c);
  const size_t row = size_t(image_w) * 4;  // floats per image row
  // this rank's bands: r, r + W, r + 2W, ... ; their rows in band order
  std::vector<std::pair<int, int>> mine;  // (first row, rows)
  size_t rows = 0;
  for (int b = I->rank; b < bt; b += W) {
    const int y0 = band_row(b, bt, image_h), y1 = band_row(b + 1, bt, image_h);
    mine.emplace_back(y0, y1 - y0);
    rows += size_t(y1 - y0);
  }
  // The eye rays of U's pixels only: a ray outside every box's footprint
  // misses the whole domain list (the reference's ISector drops it at the
  // top level), so it is counted as a traced radiance ray and not launched.
  // A pixel's samples stay consecutive in one wave (film_runs sums them in
  // order), so the film's bits match the full frame's when spp | 64; other
  // spp trace the bands whole.
  const char* ce = std::getenv("SPRAY_IMAGE_CULL");
  const bool cull = 64 % spp == 0 && !(ce && ce[0] == '0');
  if (cull) {
    r = prepare_image(I, cam, image_w, image_h, bands);
    if (r) return r;
  }
  const size_t n = cull ? size_t(I->ti.npix) * size_t(spp) : rows * size_t(image_w) * size_t(spp);
  I->nev = 0;
  I->tr->serial_begin();
  r = grow(I, I->crays, n * 32 + 32);
  if (!r) r = grow(I, I->cpix, n * 4 + 4);
  if (!r) r = grow(I, I->csam, n * 4 + 4);
  if (!r) r = mark(I, 0);
  if (cull) {
    if (!r && n) {
      CamFrame F{};
      for (int k = 0; k < 14; ++k) F.cam[k] = cam[k];
      F.image_w = image_w;
      F.spp = spp;
      if (launch_cam_eye_rays(s, I->ti, F, I->crays.as<spray_rt_ray>(), I->cpix.as<int32_t>(),
                              I->csam.as<int32_t>()) != hipSuccess)
        r = fail(c, SPRAY_RT_ERR_HIP, "eye rays");
    }
  } else {
    size_t off = 0;
    for (const auto& bnd : mine) {  // eye rays, (pixel, sample) seeds: any split, the same bits
      if (r || !bnd.second) continue;
      if (launch_eye_rays_insitu(s, cam, image_w, spp, 0, 0, image_w, 0, bnd.first, image_w,
                                 bnd.second, I->crays.as<spray_rt_ray>() + off,
                                 I->cpix.as<int32_t>() + off, I->csam.as<int32_t>() + off) !=
          hipSuccess)
        r = fail(c, SPRAY_RT_ERR_HIP, "eye rays");
      off += size_t(bnd.second) * size_t(image_w) * size_t(spp);
    }
  }
  // the rows to rank 0 (HdrImage::composite, image.h:167-181: an MPI_Reduce
  // SUM of disjoint pixels in the reference; here each rank's rows alone):
  // bands = 1 -> rank order is row order, so rank 0 receives straight into
  // its image; else the bands are packed and unpacked by 2-D copies
  auto gather = [&]() -> int {
    if (W == 1) return SPRAY_RT_OK;
    std::vector<size_t> sb(size_t(W), 0), rb(size_t(W), 0);
    if (cull) {
      // the RGB of the U pixels only (the film writes nothing else): rank k
      // packs its table's pixels, rank 0 unpacks the others' in rank order
      for (int k = 1; k < W; ++k) rb[size_t(k)] = I->rank == 0 ? size_t(I->img_counts[size_t(k)]) * 12 : 0;
      sb[0] = I->rank == 0 ? 0 : size_t(I->ti.npix) * 12;  // rank 0: nothing to itself
      GROW(I->gpack, I->rank == 0 ? size_t(I->tg.npix) * 12 + 16 : sb[0] + 16);
      float* pk = I->gpack.as<float>();
      if (I->rank != 0) HIPCHK(c, launch_pack_rgb(s, I->ti, image_w, image, pk));
      COMM(I->tr->alltoallv(I, pk, sb.data(), pk, rb.data(), true));
      if (I->rank == 0) HIPCHK(c, launch_unpack_rgb(s, I->tg, image_w, pk, image));
      return SPRAY_RT_OK;
    }
    std::vector<size_t> rrows(size_t(W), 0);  // rows of each rank
    for (int b = 0; b < bt; ++b)
      rrows[size_t(b % W)] += size_t(band_row(b + 1, bt, image_h) - band_row(b, bt, image_h));
    const size_t mine_b = rows * row * 4;
    sb[0] = mine_b;
    if (I->rank == 0)
      for (int k = 0; k < W; ++k) rb[size_t(k)] = rrows[size_t(k)] * row * 4;
    if (bands == 1) {
      float* base = image + size_t(mine.front().first) * row;
      COMM(I->tr->alltoallv(I, base, sb.data(), image, rb.data(), true));
      return SPRAY_RT_OK;
    }
    const size_t band_b = size_t(band_row(1, bt, image_h)) * row * 4;  // uniform bands only
    for (int b = 0; b < bt; ++b)
      if (size_t(band_row(b + 1, bt, image_h) - band_row(b, bt, image_h)) * row * 4 != band_b)
        return fail(c, SPRAY_RT_ERR_ARG, "interleaved bands need %d | %d rows", bt, image_h);
    const size_t total = size_t(image_h) * row * 4;
    GROW(I->gpack, I->rank == 0 ? total : mine_b);
    char* pk = I->gpack.as<char>();
    // band k of this rank sits at row (rank + k W) * band rows
    if (I->rank != 0) HIPCHK(c, launch_bands_copy(s, image, pk, W, bands, band_b, I->rank, 1, 1));
    COMM(I->tr->alltoallv(I, pk, sb.data(), pk, rb.data(), true));
    if (I->rank == 0)  // rank k's segment: its bands, in order
      HIPCHK(c, launch_bands_copy(s, image, pk, W, bands, band_b, 1, W - 1, 0));
    return SPRAY_RT_OK;
  };
  if (!r)
    r = trace_local(I, P, I->crays.as<spray_rt_ray>(), I->cpix.as<int32_t>(),
                    I->csam.as<int32_t>(), n, spp, image, rec, totals, gather);
  if (!r && cull && totals)  // the group's culled eye rays: every pixel outside U
    totals[0] += (uint64_t(image_w) * uint64_t(image_h) - I->img_upix) * uint64_t(spp);
  flush_phases(I, 1);
  I->tr->serial_end();
  return r;
}

int spray_rt_insitu_partition_view(const float* boxes, int n, const float cam[14], int nranks,
                                   int* owner) {
  if (!boxes || !cam || !owner || n < 0 || nranks <= 0) return SPRAY_RT_ERR_ARG;
  fp::Proj pj;
  if (!fp::make_proj(cam, &pj)) return SPRAY_RT_ERR_ARG;
  fp::partition_view(boxes, n, pj, nranks, owner);
  return SPRAY_RT_OK;
}

int spray_rt_camera_box_rows(const float cam[14], int image_w, int image_h, const float box[6],
                             int* x0, int* x1) {
  if (!cam || !box || !x0 || !x1 || image_w <= 0 || image_h <= 0) return -1;
  fp::Proj pj;
  if (!fp::make_proj(cam, &pj)) return -1;
  fp::Rows rows(static_cast<size_t>(image_h));
  const int k = fp::box_rows(pj, box, image_w, image_h, rows);
  for (int y = 0; y < image_h; ++y) {
    const auto& r = rows[size_t(y)];
    x0[y] = k == 2 ? 0 : (r.empty() ? image_w : r.front().first);
    x1[y] = k == 2 ? image_w - 1 : (r.empty() ? -1 : r.back().second);
  }
  return k;
}

int spray_rt_camera_shadow_boxes(const float box[6], const float scene[6], const float light[3],
                                 int k, float* out) {
  if (!box || !scene || !light || !out || k <= 0) return -2;
  return fp::shadow_boxes(box, scene, light, k, out);
}

int spray_rt_insitu_set_timing(spray_rt_insitu_t I, int on) {
  if (!I) return SPRAY_RT_ERR_ARG;
  I->timing = on != 0;
  return SPRAY_RT_OK;
}

int spray_rt_insitu_phase_times(spray_rt_insitu_t I, double out_ms[9], int* nphases) {
  if (!I || !out_ms) return SPRAY_RT_ERR_ARG;
  for (int k = 0; k < 9; ++k) {
    out_ms[k] = I->phase_ms[k];
    I->phase_ms[k] = 0.0;
  }
  if (nphases) *nphases = I->nph;
  return SPRAY_RT_OK;
}

int spray_rt_insitu_composite(spray_rt_insitu_t I, float* image, size_t nfloats) {
  if (!I) return SPRAY_RT_ERR_ARG;
  if (!image || !is_device_ptr(image))
    return fail(I->ctx, SPRAY_RT_ERR_ARG, "composite needs a device image");
  HIPCHK(I->ctx, hipSetDevice(I->ctx->device));
  if (I->world == 1) return SPRAY_RT_OK;
  return I->tr->reduce_f32(I, image, nfloats, 0);
}

int spray_rt_insitu_stats(spray_rt_insitu_t I, unsigned long long out[6]) {
  if (!I || !out) return SPRAY_RT_ERR_ARG;
  for (int k = 0; k < 6; ++k) out[k] = I->st[k];
  return SPRAY_RT_OK;
}

int spray_rt_insitu_collective_log(spray_rt_insitu_t I, uint64_t* out, size_t cap, size_t* n,
                                   int clear) {
  if (!I || !n || (cap && !out)) return SPRAY_RT_ERR_ARG;
  *n = size_t(I->clog_total);
  const size_t m = std::min(cap, I->clog.size());
  if (m) std::memcpy(out, I->clog.data(), m * sizeof(uint64_t));
  if (clear) {
    I->clog.clear();
    I->clog_total = 0;
  }
  return SPRAY_RT_OK;
}

}  // extern "C"
