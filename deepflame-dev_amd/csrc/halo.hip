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
// Exchange plans: which rows are packed (send entries) and where the received values land (receive entries),
// grouped per peer. The full plans carry every processor face; the even-odd solver's one-colour plans
// (Plan::colour[k], round 6) carry only the faces whose sending cell has colour k -- the half-row pass after the
// exchange reads exactly those (a colour-0 row gathers colour-1 values and vice versa), so every BiCGStab
// exchange moves half the bytes. Every processor face joins cells of opposite colours (build_ell checks it
// across ranks), so what one side sends for colour k is what the other side expects for its colour 1 - k, in
// the same canonical face order.
//
// Channels: channel 0 serves the main stream (and its overlapped comm stream), channel 1 the time step's side
// stream (chemistry + YEqn front + EEqn scheme terms beside the UEqn, capi.cpp) -- its own communicator
// (ncclCommSplit of the first) and buffers, so the two streams' exchanges never interleave on one communicator
// and never share a send buffer. Each channel's operations are issued in the same host order on every rank.
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
  // per peer i: send scnt[i] doubles from sbuf+soff[i], receive rcnt[i] doubles into rbuf+roff[i]
  virtual void sendrecv(Ctx& x, hipStream_t st, const double* sbuf, double* rbuf, const std::vector<int>& peers,
                        const std::vector<long>& soff, const std::vector<long>& scnt, const std::vector<long>& roff,
                        const std::vector<long>& rcnt) = 0;
  virtual void allgather(hipStream_t st, const double* s, double* r, long count) = 0;
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
                const std::vector<long>& soff, const std::vector<long>& scnt, const std::vector<long>& roff,
                const std::vector<long>& rcnt) override {
    DFMI_NCCL(ncclGroupStart());
    for (size_t i = 0; i < peers.size(); ++i) {
      if (scnt[i]) DFMI_NCCL(ncclSend(sbuf + soff[i], scnt[i], ncclDouble, peers[i], comm, st));
      if (rcnt[i]) DFMI_NCCL(ncclRecv(rbuf + roff[i], rcnt[i], ncclDouble, peers[i], comm, st));
    }
    DFMI_NCCL(ncclGroupEnd());
  }
  void allgather(hipStream_t st, const double* s, double* r, long count) override {
    DFMI_NCCL(ncclAllGather(s, r, count, ncclDouble, comm, st));
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
std::map<std::pair<int, int>, std::shared_ptr<Hub>> g_hubs;   // (hub id, channel)

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
                const std::vector<long>& soff, const std::vector<long>&, const std::vector<long>& roff,
                const std::vector<long>& rcnt) override {
    Hub& h = *hub;
    h.sb[rank] = sbuf; h.peers[rank] = peers; h.off[rank] = soff;
    DFMI_HIP(hipEventRecord(h.ev1[rank], st));
    h.barrier();
    for (size_t i = 0; i < peers.size(); ++i) {
      const int q = peers[i];
      const auto& qp = h.peers[q];
      const long j = std::find(qp.begin(), qp.end(), rank) - qp.begin();
      DFMI_CHECK(j < (long)qp.size(), "halo: peer does not list this rank");
      if (rcnt[i] == 0) continue;
      DFMI_HIP(hipStreamWaitEvent(st, h.ev1[q], 0));
      DFMI_HIP(hipMemcpyAsync(rbuf + roff[i], h.sb[q] + h.off[q][j], rcnt[i] * sizeof(double), hipMemcpyDeviceToDevice,
                              st));
    }
    finish(st);
  }
  void allgather(hipStream_t st, const double* s, double* r, long count) override {
    Hub& h = *hub;
    h.sb[rank] = s;
    DFMI_HIP(hipEventRecord(h.ev1[rank], st));
    h.barrier();
    for (int q = 0; q < h.n; ++q) {
      if (q != rank) DFMI_HIP(hipStreamWaitEvent(st, h.ev1[q], 0));
      DFMI_HIP(hipMemcpyAsync(r + (long)q * count, h.sb[q], count * sizeof(double), hipMemcpyDeviceToDevice, st));
    }
    finish(st);
  }
};

// One exchange plan: send entries (rows packed from the source arrays) and receive entries (indices the values
// land at), each grouped per peer in canonical face order. Pack layout per peer block: [component][entry].
struct Plan {
  int ns = 0, nr = 0;
  DevBuf<int> sidx, soff, scnt;   // per send entry: source row; its peer block's first entry and entry count
  DevBuf<int> ridx, roff, rcnt;   // per receive entry: destination index (slot, or halo index); block as above
  std::vector<long> ps_off, ps_cnt, pr_off, pr_cnt;   // per peer: first entry / entries
  void build(const std::vector<std::vector<int>>& s, const std::vector<std::vector<int>>& r, hipStream_t st) {
    std::vector<int> si, so, sc, ri, ro, rc;
    ps_off.clear(); ps_cnt.clear(); pr_off.clear(); pr_cnt.clear();
    for (size_t i = 0; i < s.size(); ++i) {
      ps_off.push_back((long)si.size()); ps_cnt.push_back((long)s[i].size());
      for (int v : s[i]) { so.push_back((int)ps_off.back()); sc.push_back((int)s[i].size()); si.push_back(v); }
      pr_off.push_back((long)ri.size()); pr_cnt.push_back((long)r[i].size());
      for (int v : r[i]) { ro.push_back((int)pr_off.back()); rc.push_back((int)r[i].size()); ri.push_back(v); }
    }
    ns = (int)si.size(); nr = (int)ri.size();
    auto up = [&](DevBuf<int>& d, std::vector<int>& v) { if (v.empty()) v.push_back(0); d.upload(v, st); };
    up(sidx, si); up(soff, so); up(scnt, sc); up(ridx, ri); up(roff, ro); up(rcnt, rc);
  }
};

struct Channel {
  Transport* tr = nullptr;
  DevBuf<double> sbuf, rbuf;
  std::vector<long> soff, scnt, roff, rcnt;   // per peer, in doubles, for the current exchange
  ~Channel() { delete tr; }
};

struct Halo {
  Channel ch[2];                            // 0: main stream, 1: the time step's side stream
  std::vector<int> peers;                   // ascending
  std::vector<long> pf_off, pf_cnt;         // per peer: first halo index, faces
  std::vector<int> h_cells;                 // per halo index: the local cell across the face
  Plan slots, vec, split, colour[2];        // full (to slots / to halo entries), even-odd rows, one colour
  bool have_split = false;
  // overlapped exchanges (halo_begin / halo_end): pack, transfer and unpack run on their own stream
  hipStream_t cs = nullptr;
  hipEvent_t ev_start = nullptr, ev_done = nullptr;
  bool pending = false;
  ~Halo() {
    if (cs) { (void)hipStreamSynchronize(cs); (void)hipStreamDestroy(cs); }
    if (ev_start) (void)hipEventDestroy(ev_start);
    if (ev_done) (void)hipEventDestroy(ev_done);
  }
};

void halo_destroy(Halo* h) { delete h; }
Ctx::~Ctx() {
  if (stream) (void)hipStreamSynchronize(stream);   // no posted convergence record in flight into freed memory
  if (stream2) (void)hipStreamSynchronize(stream2);
  halo_destroy(halo);
  halo = nullptr;
  if (stream2) (void)hipStreamDestroy(stream2);
  if (ev_fork) (void)hipEventDestroy(ev_fork);
  if (ev_join) (void)hipEventDestroy(ev_join);
  if (ev_u) (void)hipEventDestroy(ev_u);
  if (ev_e) (void)hipEventDestroy(ev_e);
  if (ev_cw) (void)hipEventDestroy(ev_cw);
  if (ev_th) (void)hipEventDestroy(ev_th);
  if (ev_tr) (void)hipEventDestroy(ev_tr);
}

bool halo_active(const Ctx& x) { return x.halo != nullptr && x.H > 0; }

namespace {

constexpr int MAXK = 48;
struct PackArgs { const double* src[MAXK]; double* dst[MAXK]; };

__global__ void k_pack(int n, int K, PackArgs a, const int* __restrict__ sidx, const int* __restrict__ soff,
                       const int* __restrict__ scnt, double* __restrict__ sbuf) {
  const int e = blockIdx.x * blockDim.x + threadIdx.x;
  const int k = blockIdx.y;
  if (e >= n) return;
  const long o = soff[e];
  sbuf[(long)K * o + (long)k * scnt[e] + (e - o)] = a.src[k][sidx[e]];
}
__global__ void k_unpack(int n, int K, PackArgs a, const int* __restrict__ ridx, int base, const int* __restrict__ roff,
                         const int* __restrict__ rcnt, const double* __restrict__ rbuf) {
  const int e = blockIdx.x * blockDim.x + threadIdx.x;
  const int k = blockIdx.y;
  if (e >= n) return;
  const long o = roff[e];
  a.dst[k][base + ridx[e]] = rbuf[(long)K * o + (long)k * rcnt[e] + (e - o)];
}

// the channel a stream's exchanges use: the side stream has its own (capi.cpp dfmi_time_step)
int channel_of(const Ctx& x, hipStream_t st) {
  return (x.stream2 != nullptr && st == x.stream2 && x.halo->ch[1].tr != nullptr) ? 1 : 0;
}

// pack, send/receive and unpack on stream st (x.stream: in order with the compute; the comm stream:
// overlapped, the kernel timers are not used there)
void exchange(Ctx& x, const std::vector<const double*>& src, const std::vector<double*>& dst, const Plan& pl, int base,
              hipStream_t st) {
  Halo& h = *x.halo;
  const int chan = channel_of(x, st);
  Channel& c = h.ch[chan];
  const bool timed = st == x.stream;
  const int K = (int)src.size();
  for (int k0 = 0; k0 < K; k0 += MAXK) {
    const int kk = std::min(MAXK, K - k0);
    PackArgs a{};
    for (int k = 0; k < kk; ++k) { a.src[k] = src[k0 + k]; a.dst[k] = dst[k0 + k]; }
    if (pl.ns > 0) {
      KScope _ks(x, timed ? "k_halo_pack" : nullptr);
      hipLaunchKernelGGL(k_pack, dim3(blocks_for(pl.ns, 256), kk), dim3(256), 0, st, pl.ns, kk, a, pl.sidx.p, pl.soff.p,
                         pl.scnt.p, c.sbuf.p);
    }
    DFMI_HIP(hipGetLastError());
    const size_t np = h.peers.size();
    c.soff.resize(np); c.scnt.resize(np); c.roff.resize(np); c.rcnt.resize(np);
    for (size_t i = 0; i < np; ++i) {
      c.soff[i] = (long)kk * pl.ps_off[i]; c.scnt[i] = (long)kk * pl.ps_cnt[i];
      c.roff[i] = (long)kk * pl.pr_off[i]; c.rcnt[i] = (long)kk * pl.pr_cnt[i];
    }
    if (x.comm.on) {
      // the side stream's exchanges (channel 1) are reported as their own points
      auto& e = x.comm.pts[(x.comm.tag.empty() ? std::string("halo") : x.comm.tag) + (chan ? " @side" : "")];
      hipEvent_t ea = x.comm.next(), eb = x.comm.next();
      DFMI_HIP(hipEventRecord(ea, st));
      c.tr->sendrecv(x, st, c.sbuf.p, c.rbuf.p, h.peers, c.soff, c.scnt, c.roff, c.rcnt);
      DFMI_HIP(hipEventRecord(eb, st));
      e.ev.push_back({ea, eb});
      e.calls += 1;
      for (long v : c.scnt) e.bytes += 8.0 * (double)v;
    } else {
      c.tr->sendrecv(x, st, c.sbuf.p, c.rbuf.p, h.peers, c.soff, c.scnt, c.roff, c.rcnt);
    }
    if (pl.nr > 0) {
      KScope _ks(x, timed ? "k_halo_unpack" : nullptr);
      hipLaunchKernelGGL(k_unpack, dim3(blocks_for(pl.nr, 256), kk), dim3(256), 0, st, pl.nr, kk, a, pl.ridx.p, base,
                         pl.roff.p, pl.rcnt.p, c.rbuf.p);
    }
    DFMI_HIP(hipGetLastError());
  }
}

// the items' components and the plan they share
const Plan& collect(Ctx& x, const HaloItem* items, int n, std::vector<const double*>& src, std::vector<double*>& dst,
                    int& base) {
  Halo& h = *x.halo;
  const bool slots = n > 0 ? items[0].to_slots : true, split = n > 0 && items[0].split;
  const int colour = n > 0 ? items[0].colour : -1;
  for (int i = 0; i < n; ++i) {
    DFMI_CHECK(items[i].to_slots == slots, "halo_update: mixed slot / vector destinations");
    DFMI_CHECK(items[i].split == split && items[i].colour == colour, "halo_update: mixed cell / even-odd row orders");
    for (int k = 0; k < items[i].ncomp; ++k) {
      src.push_back(items[i].cell + k * items[i].cstride);
      dst.push_back(items[i].dst + k * items[i].dstride);
    }
  }
  DFMI_CHECK(!split || h.have_split, "halo: split vectors before halo_set_split");
  DFMI_CHECK(colour < 0 || (split && !slots && colour <= 1), "halo: a one-colour exchange is an even-odd vector exchange");
  base = slots ? 0 : x.C;
  if (slots) return h.slots;
  if (!split) return h.vec;
  return colour < 0 ? h.split : h.colour[colour];
}

}  // namespace

void halo_update(Ctx& x, const HaloItem* items, int n) {
  if (!halo_active(x)) return;
  DFMI_CHECK(!x.halo->pending || channel_of(x, x.stream) == 1, "halo_update while an overlapped exchange is in flight");
  std::vector<const double*> src;
  std::vector<double*> dst;
  int base = 0;
  const Plan& pl = collect(x, items, n, src, dst, base);
  if (!src.empty()) exchange(x, src, dst, pl, base, x.stream);
}

bool halo_overlap(const Ctx& x) { return halo_active(x) && x.on("halo.overlap"); }

// overlapped exchange: everything queued on x.stream so far (the values to send) completes before the
// comm stream packs; the compute stream may run work that reads no halo entry (and writes none of the
// sent vectors) until halo_end joins the comm stream back
void halo_begin(Ctx& x, const HaloItem* items, int n) {
  Halo& h = *x.halo;
  DFMI_CHECK(!h.pending, "halo_begin: an overlapped exchange is already in flight");
  DFMI_CHECK(channel_of(x, x.stream) == 0, "halo_begin: overlapped exchanges belong to the main stream");
  if (!h.cs) {
    DFMI_HIP(hipStreamCreateWithFlags(&h.cs, hipStreamNonBlocking));
    DFMI_HIP(hipEventCreateWithFlags(&h.ev_start, hipEventDisableTiming));
    DFMI_HIP(hipEventCreateWithFlags(&h.ev_done, hipEventDisableTiming));
  }
  std::vector<const double*> src;
  std::vector<double*> dst;
  int base = 0;
  const Plan& pl = collect(x, items, n, src, dst, base);
  DFMI_HIP(hipEventRecord(h.ev_start, x.stream));
  DFMI_HIP(hipStreamWaitEvent(h.cs, h.ev_start, 0));
  if (!src.empty()) exchange(x, src, dst, pl, base, h.cs);
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
  Transport* tr = x.halo->ch[channel_of(x, x.stream)].tr;
  if (!x.comm.on) { tr->allgather(x.stream, send, recv, count); return; }
  auto& e = x.comm.pts["allgather " + (x.comm.tag.empty() ? std::string("-") : x.comm.tag)];
  hipEvent_t a = x.comm.next(), b = x.comm.next();
  DFMI_HIP(hipEventRecord(a, x.stream));
  tr->allgather(x.stream, send, recv, count);
  DFMI_HIP(hipEventRecord(b, x.stream));
  e.ev.push_back({a, b});
  e.calls += 1;
  e.bytes += 8.0 * (double)count;
}

// {"point": {"calls": n, "bytes": b, "ms": t}, ...} of the exchanges since dfmi_comm_timer (synchronises)
std::string comm_report(Ctx& x) {
  DFMI_HIP(hipStreamSynchronize(x.stream));
  if (x.stream2) DFMI_HIP(hipStreamSynchronize(x.stream2));
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
  std::vector<std::vector<int>> s_cells, r_slots, r_halo;
  std::vector<int> cells;
  x.h_hidx.assign(x.B, -1);
  h.peers.clear(); h.pf_off.clear(); h.pf_cnt.clear();
  for (auto& kv : by_peer) {
    auto& v = kv.second;
    std::sort(v.begin(), v.end(), [](const PP& l, const PP& r) { return l.key0 != r.key0 ? l.key0 < r.key0 : l.key1 < r.key1; });
    const long o = (long)cells.size();
    s_cells.emplace_back(); r_slots.emplace_back(); r_halo.emplace_back();
    for (auto& pp : v) {
      for (int i = 0; i < x.psize[pp.patch]; ++i) {
        const int b = x.poff[pp.patch] + i;   // primary (neighbour-value) slot
        x.h_hidx[b] = (int)cells.size();
        r_halo.back().push_back((int)cells.size());
        cells.push_back(x.h_bfc[b]);
        s_cells.back().push_back(x.h_bfc[b]);
        r_slots.back().push_back(b);
      }
    }
    h.peers.push_back(kv.first); h.pf_off.push_back(o); h.pf_cnt.push_back((long)cells.size() - o);
  }
  x.H = (int)cells.size();
  h.h_cells = cells;
  h.slots.build(s_cells, r_slots, x.stream);
  h.vec.build(s_cells, r_halo, x.stream);
  h.have_split = false;
  for (Channel& c : h.ch) {   // sized once: peers may still read them asynchronously
    c.sbuf.alloc((size_t)std::max(x.H, 1) * MAXK);
    c.rbuf.alloc((size_t)std::max(x.H, 1) * MAXK);
  }
  DFMI_HIP(hipStreamSynchronize(x.stream));
  // verify both sides of every interface agree on the face count (a mismatch would hang RCCL)
  const int R = x.nranks;
  DevBuf<double> s, r;
  std::vector<double> cnt(R, 0.0), all((size_t)R * R);
  for (size_t i = 0; i < h.peers.size(); ++i) cnt[h.peers[i]] = (double)h.pf_cnt[i];
  s.upload(cnt, x.stream);
  r.alloc((size_t)R * R);
  h.ch[0].tr->allgather(x.stream, s.p, r.p, R);
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

// The even-odd layout's plans (after build_ell decided it): send value[eo_pos[cell]]; all faces, and per colour k
// the faces whose local cell has colour k (sent) / colour 1 - k (received: the peer's cell has colour k)
void halo_set_split(Ctx& x) {
  Halo& h = *x.halo;
  const std::vector<int>& pos = x.ell.h_eo_pos;
  DFMI_CHECK(x.ell.eo && (int)pos.size() == x.C, "halo_set_split: no even-odd layout");
  const int ne = x.ell.ne;
  std::vector<std::vector<int>> s_all, r_all, s_k[2], r_k[2];
  for (size_t i = 0; i < h.peers.size(); ++i) {
    s_all.emplace_back(); r_all.emplace_back();
    for (int k = 0; k < 2; ++k) { s_k[k].emplace_back(); r_k[k].emplace_back(); }
    for (long e = h.pf_off[i]; e < h.pf_off[i] + h.pf_cnt[i]; ++e) {
      const int row = pos[h.h_cells[e]];
      const int col = row >= ne ? 1 : 0;
      s_all.back().push_back(row);
      r_all.back().push_back((int)e);
      s_k[col].back().push_back(row);
      r_k[1 - col].back().push_back((int)e);
    }
  }
  h.split.build(s_all, r_all, x.stream);
  for (int k = 0; k < 2; ++k) h.colour[k].build(s_k[k], r_k[k], x.stream);
  h.have_split = true;
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
  // the side stream's communicator: the same ranks, its own operation order (collective on every rank)
  auto* t2 = new RcclTransport();
  r = ncclCommSplit(t->comm, 0, rank, &t2->comm, nullptr);
  if (r != ncclSuccess) { delete t; delete t2; throw Error(std::string("ncclCommSplit: ") + ncclGetErrorString(r)); }
  delete x.halo;
  x.halo = new Halo();
  x.halo->ch[0].tr = t;
  x.halo->ch[1].tr = t2;
}

void halo_init_local(Ctx& x, int hub_id, int nranks, int rank) {
  Transport* tr[2];
  for (int c = 0; c < 2; ++c) {
    std::shared_ptr<Hub> hub;
    {
      std::lock_guard<std::mutex> l(g_hubs_m);
      auto& e = g_hubs[{hub_id, c}];
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
    tr[c] = t;
  }
  delete x.halo;
  x.halo = new Halo();
  x.halo->ch[0].tr = tr[0];
  x.halo->ch[1].tr = tr[1];
}

void rccl_unique_id(void* out) {
  ncclUniqueId id;
  DFMI_NCCL(ncclGetUniqueId(&id));
  std::memcpy(out, &id, sizeof(id));
}

}  // namespace dfmi
