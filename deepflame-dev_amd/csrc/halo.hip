// halo.hip -- processor-patch halo exchange (replaces dfNcclBase.cu:23-65 and the per-patch
// ncclSend/ncclRecv groups of correct_boundary_conditions_processor_{scalar,vector},
// dfMatrixOpBase.cu:441-485, and fvc_grad_vector_correctBC_processor, :1366-1389).
//
// Design: per exchange point ONE packed message per neighbour rank carrying every
// field component that point needs, instead of one NCCL group per field and patch. Patches to the same
// neighbour are concatenated in a canonical order both sides derive independently (sorted by the
// global-id pair of their first face), faces within a patch are in OpenFOAM's matching order.
// Send layout per peer: [component][face]. Received values land in the neighbour half of the
// processor slots ([neighbour n | internal n], createGPUSolver.H:118-123), or in the extended region
// [C, C+H) of a solver vector (the SpMV reads processor columns there).
//
// Two transports behind one interface:
//   * RCCL (ncclSend/ncclRecv in a group, ncclAllGather), one process per GPU over xGMI -- the product;
//   * in-process hub (device-to-device copies between contexts driven by host threads), so several
//     ranks can share one GPU in tests (RCCL refuses two ranks on one device).
#include "dfmi_ctx.h"
#include <rccl/rccl.h>
#include <algorithm>
#include <condition_variable>
#include <cstring>
#include <mutex>
#include <numeric>

namespace dfmi {

struct Transport {
  virtual ~Transport() = default;
  // per peer i: send cnt[i] doubles from sbuf+off[i], receive cnt[i] doubles into rbuf+off[i]
  virtual void sendrecv(Ctx& x, hipStream_t st, const double* sbuf, double* rbuf, const std::vector<int>& peers,
                        const std::vector<long>& off, const std::vector<long>& cnt) = 0;
  virtual void allgather(Ctx& x, const double* s, double* r, long count) = 0;
};

#define DFMI_NCCL(call)                                                                                      \
  do {                                                                                                       \
    ncclResult_t _r = (call);                                                                                \
    if (_r != ncclSuccess) throw Error(std::string("RCCL error ") + ncclGetErrorString(_r) + " in " #call); \
  } while (0)

struct RcclTransport : Transport {
  ncclComm_t comm = nullptr;
  ~RcclTransport() override { if (comm) (void)ncclCommDestroy(comm); }
  void sendrecv(Ctx&, hipStream_t st, const double* sbuf, double* rbuf, const std::vector<int>& peers,
                const std::vector<long>& off, const std::vector<long>& cnt) override {
    DFMI_NCCL(ncclGroupStart());
    for (size_t i = 0; i < peers.size(); ++i) {
      DFMI_NCCL(ncclSend(sbuf + off[i], cnt[i], ncclDouble, peers[i], comm, st));
      DFMI_NCCL(ncclRecv(rbuf + off[i], cnt[i], ncclDouble, peers[i], comm, st));
    }
    DFMI_NCCL(ncclGroupEnd());
  }
  void allgather(Ctx& x, const double* s, double* r, long count) override {
    DFMI_NCCL(ncclAllGather(s, r, count, ncclDouble, comm, x.stream));
  }
};

// ---- in-process hub
struct Hub {
  int n = 0;
  std::mutex m;
  std::condition_variable cv;
  int arrived = 0;
  long gen = 0;
  std::vector<const double*> sb;
  std::vector<std::vector<int>> peers;
  std::vector<std::vector<long>> off;
  std::vector<hipEvent_t> ev1, ev2;
  void barrier() {
    std::unique_lock<std::mutex> l(m);
    const long g = gen;
    if (++arrived == n) { arrived = 0; ++gen; cv.notify_all(); }
    else cv.wait(l, [&] { return gen != g; });
  }
};
std::mutex g_hubs_m;
std::map<int, std::shared_ptr<Hub>> g_hubs;

struct LocalTransport : Transport {
  std::shared_ptr<Hub> hub;
  int rank = 0;
  ~LocalTransport() override {
    (void)hipEventDestroy(hub->ev1[rank]);
    (void)hipEventDestroy(hub->ev2[rank]);
  }
  void finish(hipStream_t st) {   // nobody reuses its send buffer before every peer has copied out of it
    Hub& h = *hub;
    DFMI_HIP(hipEventRecord(h.ev2[rank], st));
    h.barrier();
    for (int q = 0; q < h.n; ++q) if (q != rank) DFMI_HIP(hipStreamWaitEvent(st, h.ev2[q], 0));
    h.barrier();
  }
  void sendrecv(Ctx&, hipStream_t st, const double* sbuf, double* rbuf, const std::vector<int>& peers,
                const std::vector<long>& off, const std::vector<long>& cnt) override {
    Hub& h = *hub;
    h.sb[rank] = sbuf; h.peers[rank] = peers; h.off[rank] = off;
    DFMI_HIP(hipEventRecord(h.ev1[rank], st));
    h.barrier();
    for (size_t i = 0; i < peers.size(); ++i) {
      const int q = peers[i];
      const auto& qp = h.peers[q];
      const long j = std::find(qp.begin(), qp.end(), rank) - qp.begin();
      DFMI_CHECK(j < (long)qp.size(), "halo: peer does not list this rank");
      DFMI_HIP(hipStreamWaitEvent(st, h.ev1[q], 0));
      DFMI_HIP(hipMemcpyAsync(rbuf + off[i], h.sb[q] + h.off[q][j], cnt[i] * sizeof(double), hipMemcpyDeviceToDevice,
                              st));
    }
    finish(st);
  }
  void allgather(Ctx& x, const double* s, double* r, long count) override {
    Hub& h = *hub;
    h.sb[rank] = s;
    DFMI_HIP(hipEventRecord(h.ev1[rank], x.stream));
    h.barrier();
    for (int q = 0; q < h.n; ++q) {
      if (q != rank) DFMI_HIP(hipStreamWaitEvent(x.stream, h.ev1[q], 0));
      DFMI_HIP(hipMemcpyAsync(r + (long)q * count, h.sb[q], count * sizeof(double), hipMemcpyDeviceToDevice, x.stream));
    }
    finish(x.stream);
  }
};

struct Halo {
  Transport* tr = nullptr;
  std::vector<int> peers;                   // ascending
  std::vector<long> pf_off, pf_cnt;         // per peer: first halo index, faces
  DevBuf<int> send_cells, recv_slots, h_off, h_cnt;   // per halo index
  std::vector<int> h_cells;                 // send_cells on the host
  DevBuf<int> send_pos;                     // eo_pos[send_cells]: rows of split (even-odd) vectors
  DevBuf<double> sbuf, rbuf;
  std::vector<long> off, cnt;               // per peer, in doubles, for the current exchange
  // overlapped exchanges (halo_begin / halo_end): pack, transfer and unpack run on their own stream
  hipStream_t cs = nullptr;
  hipEvent_t ev_start = nullptr, ev_done = nullptr;
  bool pending = false;
  ~Halo() {
    delete tr;
    if (cs) { (void)hipStreamSynchronize(cs); (void)hipStreamDestroy(cs); }
    if (ev_start) (void)hipEventDestroy(ev_start);
    if (ev_done) (void)hipEventDestroy(ev_done);
  }
};

void halo_destroy(Halo* h) { delete h; }
Ctx::~Ctx() {
  halo_destroy(halo);
  halo = nullptr;
  if (stream) (void)hipStreamSynchronize(stream);   // no posted convergence record in flight into freed memory
  if (stream2) { (void)hipStreamSynchronize(stream2); (void)hipStreamDestroy(stream2); }
  if (ev_fork) (void)hipEventDestroy(ev_fork);
  if (ev_join) (void)hipEventDestroy(ev_join);
  if (ev_u) (void)hipEventDestroy(ev_u);
  if (ev_e) (void)hipEventDestroy(ev_e);
  if (ev_cw) (void)hipEventDestroy(ev_cw);
}

bool halo_active(const Ctx& x) { return x.halo != nullptr && x.H > 0; }

namespace {

constexpr int MAXK = 48;
struct PackArgs { const double* src[MAXK]; double* dst[MAXK]; };

__global__ void k_pack(int H, int K, PackArgs a, const int* __restrict__ cells, const int* __restrict__ hoff,
                       const int* __restrict__ hcnt, double* __restrict__ sbuf) {
  const int h = blockIdx.x * blockDim.x + threadIdx.x;
  const int k = blockIdx.y;
  if (h >= H) return;
  const long o = hoff[h];
  sbuf[(long)K * o + (long)k * hcnt[h] + (h - o)] = a.src[k][cells[h]];
}
__global__ void k_unpack(int H, int K, PackArgs a, const int* __restrict__ slots, int ext_base,
                         const int* __restrict__ hoff, const int* __restrict__ hcnt, const double* __restrict__ rbuf) {
  const int h = blockIdx.x * blockDim.x + threadIdx.x;
  const int k = blockIdx.y;
  if (h >= H) return;
  const long o = hoff[h];
  const double v = rbuf[(long)K * o + (long)k * hcnt[h] + (h - o)];
  const int idx = slots ? slots[h] : ext_base + h;
  a.dst[k][idx] = v;
}

// pack, send/receive and unpack on stream st (x.stream: in order with the compute; the comm stream:
// overlapped, the kernel timers are not used there)
void exchange(Ctx& x, const std::vector<const double*>& src, const std::vector<double*>& dst, bool to_slots,
              hipStream_t st, bool split = false) {
  Halo& h = *x.halo;
  DFMI_CHECK(!split || h.send_pos.n == h.send_cells.n, "halo: split vectors before halo_set_split");
  const int* sc = split ? h.send_pos.p : h.send_cells.p;
  const bool timed = st == x.stream;
  const int K = (int)src.size();
  for (int k0 = 0; k0 < K; k0 += MAXK) {
    const int kk = std::min(MAXK, K - k0);
    PackArgs a{};
    for (int k = 0; k < kk; ++k) { a.src[k] = src[k0 + k]; a.dst[k] = dst[k0 + k]; }
    dim3 g(blocks_for(x.H, 256), kk);
    {
      KScope _ks(x, timed ? "k_halo_pack" : nullptr);
      hipLaunchKernelGGL(k_pack, g, dim3(256), 0, st, x.H, kk, a, sc, h.h_off.p, h.h_cnt.p, h.sbuf.p);
    }
    DFMI_HIP(hipGetLastError());
    h.off.resize(h.peers.size()); h.cnt.resize(h.peers.size());
    for (size_t i = 0; i < h.peers.size(); ++i) { h.off[i] = (long)kk * h.pf_off[i]; h.cnt[i] = (long)kk * h.pf_cnt[i]; }
    if (x.comm.on) {
      auto& e = x.comm.pts[x.comm.tag.empty() ? std::string("halo") : x.comm.tag];
      hipEvent_t a = x.comm.next(), b = x.comm.next();
      DFMI_HIP(hipEventRecord(a, st));
      h.tr->sendrecv(x, st, h.sbuf.p, h.rbuf.p, h.peers, h.off, h.cnt);
      DFMI_HIP(hipEventRecord(b, st));
      e.ev.push_back({a, b});
      e.calls += 1;
      for (long c : h.cnt) e.bytes += 8.0 * (double)c;
    } else {
      h.tr->sendrecv(x, st, h.sbuf.p, h.rbuf.p, h.peers, h.off, h.cnt);
    }
    {
      KScope _ks(x, timed ? "k_halo_unpack" : nullptr);
      hipLaunchKernelGGL(k_unpack, g, dim3(256), 0, st, x.H, kk, a, to_slots ? h.recv_slots.p : nullptr, x.C, h.h_off.p,
                         h.h_cnt.p, h.rbuf.p);
    }
    DFMI_HIP(hipGetLastError());
  }
}

void collect(const HaloItem* items, int n, std::vector<const double*>& src, std::vector<double*>& dst, bool& slots,
             bool& split) {
  slots = true;
  split = false;
  for (int i = 0; i < n; ++i) {
    if (i == 0) { slots = items[i].to_slots; split = items[i].split; }
    DFMI_CHECK(items[i].to_slots == slots, "halo_update: mixed slot / vector destinations");
    DFMI_CHECK(items[i].split == split, "halo_update: mixed cell / even-odd row orders");
    for (int k = 0; k < items[i].ncomp; ++k) {
      src.push_back(items[i].cell + k * items[i].cstride);
      dst.push_back(items[i].dst + k * items[i].dstride);
    }
  }
}

}  // namespace

void halo_update(Ctx& x, const HaloItem* items, int n) {
  if (!halo_active(x)) return;
  DFMI_CHECK(!x.halo->pending, "halo_update while an overlapped exchange is in flight");
  std::vector<const double*> src;
  std::vector<double*> dst;
  bool slots = true, split = false;
  collect(items, n, src, dst, slots, split);
  if (!src.empty()) exchange(x, src, dst, slots, x.stream, split);
}

bool halo_overlap(const Ctx& x) { return halo_active(x) && x.halo_overlap; }

// overlapped exchange: everything queued on x.stream so far (the values to send) completes before the
// comm stream packs; the compute stream may run work that reads no halo entry (and writes none of the
// sent vectors) until halo_end joins the comm stream back
void halo_begin(Ctx& x, const HaloItem* items, int n) {
  Halo& h = *x.halo;
  DFMI_CHECK(!h.pending, "halo_begin: an overlapped exchange is already in flight");
  if (!h.cs) {
    DFMI_HIP(hipStreamCreateWithFlags(&h.cs, hipStreamNonBlocking));
    DFMI_HIP(hipEventCreateWithFlags(&h.ev_start, hipEventDisableTiming));
    DFMI_HIP(hipEventCreateWithFlags(&h.ev_done, hipEventDisableTiming));
  }
  std::vector<const double*> src;
  std::vector<double*> dst;
  bool slots = true, split = false;
  collect(items, n, src, dst, slots, split);
  DFMI_HIP(hipEventRecord(h.ev_start, x.stream));
  DFMI_HIP(hipStreamWaitEvent(h.cs, h.ev_start, 0));
  if (!src.empty()) exchange(x, src, dst, slots, h.cs, split);
  DFMI_HIP(hipEventRecord(h.ev_done, h.cs));
  h.pending = true;
}

void halo_end(Ctx& x) {
  Halo& h = *x.halo;
  DFMI_CHECK(h.pending, "halo_end without halo_begin");
  DFMI_HIP(hipStreamWaitEvent(x.stream, h.ev_done, 0));
  h.pending = false;
}

void halo_allgather(Ctx& x, const double* send, double* recv, long count) {
  DFMI_CHECK(x.halo && x.nranks > 1, "halo_allgather without a communicator");
  if (!x.comm.on) { x.halo->tr->allgather(x, send, recv, count); return; }
  auto& e = x.comm.pts["allgather " + (x.comm.tag.empty() ? std::string("-") : x.comm.tag)];
  hipEvent_t a = x.comm.next(), b = x.comm.next();
  DFMI_HIP(hipEventRecord(a, x.stream));
  x.halo->tr->allgather(x, send, recv, count);
  DFMI_HIP(hipEventRecord(b, x.stream));
  e.ev.push_back({a, b});
  e.calls += 1;
  e.bytes += 8.0 * (double)count;
}

// {"point": {"calls": n, "bytes": b, "ms": t}, ...} of the exchanges since dfmi_comm_timer (synchronises)
std::string comm_report(Ctx& x) {
  DFMI_HIP(hipStreamSynchronize(x.stream));
  if (x.halo && x.halo->cs) DFMI_HIP(hipStreamSynchronize(x.halo->cs));
  std::string out = "{";
  bool first = true;
  for (auto& kv : x.comm.pts) {
    double ms = 0.0;
    for (auto& pr : kv.second.ev) {
      float t = 0.f;
      DFMI_HIP(hipEventElapsedTime(&t, pr.first, pr.second));
      ms += t;
    }
    char buf[256];
    std::snprintf(buf, sizeof buf, "\"calls\": %ld, \"bytes\": %.0f, \"ms\": %.6f}", kv.second.calls, kv.second.bytes, ms);
    out += (first ? "\"" : ", \"") + kv.first + "\": {" + buf;
    first = false;
  }
  return out + "}";
}

// Exchange lists from the processor patches (called once the communicator exists).
void halo_setup(Ctx& x) {
  Halo& h = *x.halo;
  struct PP { int patch; long key0, key1; };
  std::map<int, std::vector<PP>> by_peer;
  int pf = 0;   // running index into procCols (processor faces in patch order)
  for (int p = 0; p < x.P; ++p) {
    if (x.pkind[p] != 2) continue;
    const int n = x.psize[p];
    DFMI_CHECK(x.peer[p] >= 0 && x.peer[p] < x.nranks && x.peer[p] != x.rank,
               "processor patch " + std::to_string(p) + " has no valid neighbour rank");
    DFMI_CHECK((int)x.h_proc_cols.size() >= pf + n, "procCols shorter than the processor faces");
    long a = 0, b = 0;
    if (n > 0) {
      a = (long)x.global_offset + x.h_bfc[x.poff[p]];
      b = x.h_proc_cols[pf];
    }
    by_peer[x.peer[p]].push_back({p, std::min(a, b), std::max(a, b)});
    pf += n;
  }
  std::vector<int> cells, slots, hoff, hcnt;
  x.h_hidx.assign(x.B, -1);
  h.peers.clear(); h.pf_off.clear(); h.pf_cnt.clear();
  for (auto& kv : by_peer) {
    auto& v = kv.second;
    std::sort(v.begin(), v.end(), [](const PP& l, const PP& r) { return l.key0 != r.key0 ? l.key0 < r.key0 : l.key1 < r.key1; });
    const long o = (long)cells.size();
    for (auto& pp : v) {
      for (int i = 0; i < x.psize[pp.patch]; ++i) {
        const int b = x.poff[pp.patch] + i;   // primary (neighbour-value) slot
        x.h_hidx[b] = (int)cells.size();
        cells.push_back(x.h_bfc[b]);
        slots.push_back(b);
      }
    }
    const long c = (long)cells.size() - o;
    h.peers.push_back(kv.first); h.pf_off.push_back(o); h.pf_cnt.push_back(c);
    for (long i = 0; i < c; ++i) { hoff.push_back((int)o); hcnt.push_back((int)c); }
  }
  x.H = (int)cells.size();
  if (x.H == 0) { cells.push_back(0); slots.push_back(0); hoff.push_back(0); hcnt.push_back(1); }
  h.send_cells.upload(cells, x.stream); h.recv_slots.upload(slots, x.stream);
  h.h_cells = cells;
  h.send_pos.release();
  h.sbuf.alloc((size_t)std::max(x.H, 1) * MAXK);   // sized once: peers may still read it asynchronously
  h.rbuf.alloc((size_t)std::max(x.H, 1) * MAXK);
  h.h_off.upload(hoff, x.stream); h.h_cnt.upload(hcnt, x.stream);
  DFMI_HIP(hipStreamSynchronize(x.stream));
  // verify both sides of every interface agree on the face count (a mismatch would hang RCCL)
  const int R = x.nranks;
  DevBuf<double> s, r;
  std::vector<double> cnt(R, 0.0), all((size_t)R * R);
  for (size_t i = 0; i < h.peers.size(); ++i) cnt[h.peers[i]] = (double)h.pf_cnt[i];
  s.upload(cnt, x.stream);
  r.alloc((size_t)R * R);
  h.tr->allgather(x, s.p, r.p, R);
  DFMI_HIP(hipMemcpyAsync(all.data(), r.p, all.size() * sizeof(double), hipMemcpyDeviceToHost, x.stream));
  DFMI_HIP(hipStreamSynchronize(x.stream));
  for (int q = 0; q < R; ++q)
    DFMI_CHECK(all[(size_t)x.rank * R + q] == all[(size_t)q * R + x.rank],
               "processor faces between ranks " + std::to_string(x.rank) + " and " + std::to_string(q) +
                   " disagree (" + std::to_string(all[(size_t)x.rank * R + q]) + " vs " +
                   std::to_string(all[(size_t)q * R + x.rank]) + ")");
  x.ell.ready = false;   // solver columns now include halo entries
}

std::vector<int> halo_peers_of(const Ctx& x) {
  std::vector<int> pr(std::max(x.H, 0), -1);
  if (!x.halo) return pr;
  const Halo& h = *x.halo;
  for (size_t i = 0; i < h.peers.size(); ++i)
    for (long k = 0; k < h.pf_cnt[i]; ++k) pr[h.pf_off[i] + k] = h.peers[i];
  return pr;
}

void halo_set_split(Ctx& x) {
  Halo& h = *x.halo;
  const std::vector<int>& pos = x.ell.h_eo_pos;
  DFMI_CHECK(x.ell.eo && (int)pos.size() == x.C, "halo_set_split: no even-odd layout");
  std::vector<int> sp(h.h_cells.size());
  for (size_t i = 0; i < sp.size(); ++i) sp[i] = x.H > 0 ? pos[h.h_cells[i]] : 0;
  h.send_pos.upload(sp, x.stream);
  DFMI_HIP(hipStreamSynchronize(x.stream));
}

// ---- communicator creation (used by capi.cpp)
void halo_init_rccl(Ctx& x, const void* uid, int nranks, int rank) {
  auto* t = new RcclTransport();
  ncclUniqueId id;
  static_assert(sizeof(ncclUniqueId) == 128, "RCCL unique id is 128 bytes");
  std::memcpy(&id, uid, sizeof(id));
  DFMI_HIP(hipSetDevice(x.device));
  ncclResult_t r = ncclCommInitRank(&t->comm, nranks, id, rank);
  if (r != ncclSuccess) { delete t; throw Error(std::string("ncclCommInitRank: ") + ncclGetErrorString(r)); }
  delete x.halo;
  x.halo = new Halo();
  x.halo->tr = t;
}

void halo_init_local(Ctx& x, int hub_id, int nranks, int rank) {
  std::shared_ptr<Hub> hub;
  {
    std::lock_guard<std::mutex> l(g_hubs_m);
    auto& e = g_hubs[hub_id];
    if (!e || e->n != nranks) {
      e = std::make_shared<Hub>();
      e->n = nranks;
      e->sb.assign(nranks, nullptr); e->peers.assign(nranks, {}); e->off.assign(nranks, {});
      e->ev1.assign(nranks, nullptr); e->ev2.assign(nranks, nullptr);
    }
    hub = e;
  }
  DFMI_HIP(hipEventCreateWithFlags(&hub->ev1[rank], hipEventDisableTiming));
  DFMI_HIP(hipEventCreateWithFlags(&hub->ev2[rank], hipEventDisableTiming));
  auto* t = new LocalTransport();
  t->hub = hub; t->rank = rank;
  delete x.halo;
  x.halo = new Halo();
  x.halo->tr = t;
}

void rccl_unique_id(void* out) {
  ncclUniqueId id;
  DFMI_NCCL(ncclGetUniqueId(&id));
  std::memcpy(out, &id, sizeof(id));
}

}  // namespace dfmi
