// api.hip — the C ABI of libswimhip (include/swimhip.h): configuration, device allocation, fault injection, readback.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <condition_variable>
#include <mutex>
#include <thread>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <map>
#include <string>
#include <vector>

#include <rccl/rccl.h>

#include "../../include/swimhip.h"
#include "../../include/swimhip_shard.h"
#include "../../include/swimhip_wire.h"
#include "../../include/swimhip_debug.h"
#include "engine.h"

using namespace swim;

struct Group;  // swim_config.n_gpus > 1: one handle over several row-sharded shard handles (below)

constexpr size_t GUARD = 4096;  // SWIM_GUARD: guard bytes on each side of every device allocation

struct swim_handle {
  swim_config cfg;
  Dev d;
  hipStream_t stream = nullptr;
  uint64_t tick = 0;
  std::string err;
  std::vector<void*> allocs;
  std::vector<std::pair<char*, size_t>> guards;  // SWIM_GUARD: (allocation, bytes inside the guards)
  std::vector<swim_event> host_events;
  // settings-epoch ring mirrored on the host
  uint32_t ep_from[MAX_EPOCHS], ep_loss[MAX_EPOCHS], ep_part[MAX_EPOCHS], ep_delay[MAX_EPOCHS];
  int cur_ep = 0;
  uint32_t loss = 0;
  uint32_t delay_idx = 0;                 // default mean delay (index into delays)
  std::vector<uint32_t> delays{0};        // mean delay ms of each delay index (0: none)
  bool partitioned = false;
  std::vector<uint32_t> group;
  // per-link NetworkEmulator settings: current custom settings and each link's change history (mirrored to HBM)
  std::map<uint64_t, uint32_t> link_cur;
  std::map<uint64_t, std::vector<std::pair<uint32_t, uint32_t>>> link_hist;
  size_t bytes = 0;
  std::vector<TickEvents> prof;  // SWIM_FLAG_PROFILE: one event set per tick of the current swim_step
  double prof_ms[3] = {0, 0, 0};  // accumulated k_sync_diff, k_member_tick, k_gossip_send
  uint64_t prof_diff_launches = 0;
  // row sharding (swimhip_shard.h)
  swim_shard_spec spec{};
  ncclComm_t comm = nullptr;
  unsigned long long* hcnt = nullptr;  // pinned [2W]: send then receive byte counts of the current exchange
  std::vector<uint8_t> hsend, hrecv;  // SWIM_TRANSPORT_HOST staging
  double xchg_ms = 0;                 // host time spent in the exchanges
  bool xflag = false;                 // last exchange: some shard has a gossip slot in use
  std::vector<uint8_t> joined;  // swim_join: dormant members that were started
  std::vector<uint32_t> md_cols;  // swim_update_metadata: members that own a metadata-version column
  std::vector<uint64_t> ugq;  // swim_spread_gossip queue: (member, payload) pairs for P0 of the next tick
  uint64_t* ug_dev = nullptr;  // device copy of ugq
  size_t ug_cap = 0;
  volatile uint32_t* hflag = nullptr; // host-mapped flag word written by k_tick_flag (W == 1)
  unsigned long long* xi_host_h = nullptr;  // host side of Dev::xi_host
  hipEvent_t ev_member = nullptr;
  uint64_t next_scrub = SCRUB;  // tick of the next k_s_scrub (16-bit holder entries, engine.h)
  bool no_skip = getenv("SWIM_NO_GOSSIP_SKIP") != nullptr;  // debugging aid: always run the gossip data plane
  bool no_pipe = getenv("SWIM_NO_PIPELINE") != nullptr;    // debugging aid: no early SYNC diff of the next tick
  bool no_spec = getenv("SWIM_NO_SPECULATION") != nullptr;  // debugging aid: a host wait after every member kernel
  bool gossip_idle = false;  // W == 1: no gossip slot was in use after the latest member kernel
  bool gossip_ran = false;   // W == 1: the latest tick ran the gossip plane (the next P4 may have routed receipts)
  uint64_t growths = 0;      // capacity growth steps so far (grow_caps)
  uint64_t grow_next = 0;    // grow_caps: no attempt before this tick (the last one found no room)
  // timing aid (bench.py --rehearse-shard): a slot shard alone, its peers' gossip-count deltas taken as zero without
  // any exchange (not the W-shard simulation's results)
  bool lone = getenv("SWIM_LONE_SHARD") != nullptr;
  // timing aid (SWIM_STATS): the gossip plane's work per tick on stderr (routed receipts, targets, active groups,
  // replay / slow-path sends, contact pairs, RX rows); one stream wait per tick
  bool stats = getenv("SWIM_STATS") != nullptr;
  Group* grp = nullptr;  // n_gpus > 1: every call is forwarded to the shards (d holds shard 0's constants only)
};

namespace {

#define HIPCK(expr)                                                        \
  do {                                                                     \
    hipError_t e_ = (expr);                                                \
    if (e_ != hipSuccess) {                                                \
      h->err = std::string(#expr " -> ") + hipGetErrorString(e_);          \
      return SWIM_EDEVICE;                                                 \
    }                                                                      \
  } while (0)

template <class T>
int dalloc(swim_handle* h, T** p, size_t count) {
  size_t bytes = std::max<size_t>(count, 1) * sizeof(T);
  void* q = nullptr;
  // debugging aid (SWIM_GUARD): GUARD bytes of 0x5A before and after every allocation, checked after every step
  const bool guard = getenv("SWIM_GUARD") != nullptr;
  hipError_t e = hipMalloc(&q, bytes + (guard ? 2 * GUARD : 0));
  if (e != hipSuccess) {
    h->err = "hipMalloc(" + std::to_string(bytes) + ") failed: " + hipGetErrorString(e);
    return SWIM_ENOMEM;
  }
  h->allocs.push_back(q);
  if (guard) {
    hipMemsetAsync(q, 0x5A, GUARD, h->stream);
    hipMemsetAsync((char*)q + GUARD + bytes, 0x5A, GUARD, h->stream);
    h->guards.push_back({(char*)q, bytes});
    q = (char*)q + GUARD;
  }
  h->bytes += bytes;
  // debugging aids: poison fresh allocations (all, or only allocation #SWIM_POISON_ONLY) to catch never-written state
  const char* po = getenv("SWIM_POISON_ONLY");
  if (getenv("SWIM_POISON") || (po && atoi(po) == (int)h->allocs.size() - 1)) hipMemsetAsync(q, 0xA5, bytes, h->stream);
  *p = (T*)q;
  return SWIM_OK;
}

hipError_t h2d(hipStream_t st, void* dst, const void* src, size_t bytes);

// an allocation of dalloc given back (capacity growth replaced it)
void dfree(swim_handle* h, void* p, size_t bytes) {
  auto it = std::find(h->allocs.begin(), h->allocs.end(), p);
  if (it == h->allocs.end()) return;
  h->allocs.erase(it);
  hipFree(p);
  h->bytes -= bytes;
}

// ---------------------------------------------------------------------------------------------------------------
// Capacity growth (one GPU). The gossip slot table, the receipt rings and the per-tick receipt / replay lists start
// at the config's size and grow between ticks before they can overflow: after each member kernel of a tick with the
// gossip plane active, tick_flag has published the slots in use, the largest ring fill and the previous gossip plane's
// list lengths (Dev::hflag). A structure past half (slots, rings) or a quarter (per-tick lists) of its capacity is
// reallocated larger, within the free HBM, its contents moved: slot ids, ring positions and every held bit keep their
// meaning, so the simulation is unchanged (slot ids are not observable). SWIM_NO_GROW: fixed sizes.
static int grow_caps_(swim_handle* h);
int grow_caps(swim_handle* h) {
  const int rc = grow_caps_(h);
  // a structure replaced before a later allocation failed: the device copy of Dev must name the new buffers (the old
  // ones are freed), so it is uploaded on that path too
  if (rc != SWIM_OK) (void)h2d(h->stream, (void*)h->d.self, &h->d, sizeof(Dev));
  return rc;
}
static int grow_caps_(swim_handle* h) {
  Dev& d = h->d;
  if (!d.rfill) return SWIM_OK;
  // (a row shard publishes only the ring fill and the history entries, grow_caps_shard: [0], [3..5] stay 0)
  const volatile uint32_t* f = h->hflag;
  const uint64_t used = f[0], fill = f[2], nrc = f[3], nrp = f[4], nsl = f[5], nhist = f[6];
  const uint64_t N = d.N;
  const bool gs = used > d.SPR / 2 && d.SPR < (1u << 22), gr = fill > d.BCAP / 2 && d.BCAP < (1u << 30);
  const bool grc = nrc > d.RCAP / 4 && d.RCAP < (1u << 30), grp = (nrp > d.RPCAP / 4 || nsl > d.SLOWCAP / 4) && d.RPCAP < (1u << 30);
  // the history scales with the holder states that can be reborn: the create-time rule (slots x members / 8, up to
  // 2^24) for the grown slot table, or four times the entries in use
  uint64_t hwant = d.HCAP;
  if (nhist > d.HCAP / 2) hwant = 4 * nhist;
  if (gs) hwant = std::max<uint64_t>(hwant, std::min<uint64_t>(1ull << 24, 2ull * d.SPR * N / 8));
  uint64_t hcap2 = d.HCAP;
  while (hcap2 < hwant && hcap2 < (1ull << 28)) hcap2 <<= 1;
  const bool gh = hcap2 > d.HCAP;
  if (!gs && !gr && !grc && !grp && !gh) return SWIM_OK;
  // an attempt the free HBM could not serve is not repeated every tick (each one waits for the stream): the sizes
  // that fit stay, and the next attempt is SCRUB ticks later
  if (h->tick < h->grow_next) return SWIM_OK;
  const uint64_t bytes0 = h->bytes, growths0 = h->growths;
  HIPCK(hipStreamSynchronize(h->stream));
  size_t fr = 0, tot = 0;
  HIPCK(hipMemGetInfo(&fr, &tot));
  const uint64_t reserve = 2ull << 30;
  uint64_t budget = fr > reserve ? fr - reserve : 0;
  hipStream_t st = h->stream;
  int rc;
  if (grc || grp) {  // per-tick lists: nothing in them between ticks, so no contents move
    const uint64_t rcap = grc ? std::min<uint64_t>(1ull << 30, std::max<uint64_t>(4ull * nrc, 4ull * d.RCAP)) : d.RCAP;
    const uint64_t pcap = grp ? std::min<uint64_t>(1ull << 30, 4ull * std::max<uint64_t>(d.RPCAP, std::max(nrp, nsl))) : d.RPCAP;
    const uint64_t need = (rcap - d.RCAP) * 32 + (pcap - d.RPCAP) * 16;
    if (need <= budget) {
      budget -= need;
      // every replacement is allocated before an old buffer is given back: a failed allocation leaves the handle on
      // its old (valid) buffers
      if (rcap != d.RCAP) {
        uint64_t *raw2 = nullptr, *key2 = nullptr, *keyb = nullptr;
        uint32_t *slot2 = nullptr, *slotb = nullptr;
        if ((rc = dalloc(h, &raw2, rcap)) || (rc = dalloc(h, &slot2, rcap)) || (rc = dalloc(h, &key2, rcap)) ||
            (rc = dalloc(h, &slotb, rcap)) || (rc = dalloc(h, &keyb, rcap))) {
          dfree(h, raw2, 8 * rcap), dfree(h, slot2, 4 * rcap), dfree(h, key2, 8 * rcap), dfree(h, slotb, 4 * rcap);
          return rc;
        }
        dfree(h, d.rc_raw, 8ull * d.RCAP), dfree(h, d.rc_slot, 4ull * d.RCAP), dfree(h, d.rc_key, 8ull * d.RCAP);
        dfree(h, d.rc_slot2, 4ull * d.RCAP), dfree(h, d.rc_key2, 8ull * d.RCAP);
        d.rc_raw = raw2, d.rc_slot = slot2, d.rc_key = key2, d.rc_slot2 = slotb, d.rc_key2 = keyb;
        d.RCAP = d.DCAP = (uint32_t)rcap;
      }
      if (pcap != d.RPCAP) {
        uint64_t *rp2 = nullptr, *slow2 = nullptr;
        if ((rc = dalloc(h, &rp2, pcap)) || (rc = dalloc(h, &slow2, pcap))) {
          dfree(h, rp2, 8 * pcap);
          return rc;
        }
        dfree(h, d.rp, 8ull * d.RPCAP), dfree(h, d.slow, 8ull * d.SLOWCAP);
        d.rp = rp2, d.slow = slow2;
        d.RPCAP = d.SLOWCAP = (uint32_t)pcap;
      }
    }
  }
  if (gh && 8ull * hcap2 * HREC <= budget) {  // incarnation history: a larger table, every entry re-inserted
    uint64_t* h2 = nullptr;
    const uint64_t c2 = hcap2;
    budget -= 8 * c2 * HREC;
    if ((rc = dalloc(h, &h2, c2 * HREC))) return rc;
    HIPCK(hipMemsetAsync(h2, 0, 8 * c2 * HREC, st));
    launch_hist_rehash(d.hist, d.HCAP, h2, (uint32_t)c2, st);
    HIPCK(hipStreamSynchronize(st));
    dfree(h, d.hist, 8ull * d.HCAP * HREC);
    d.hist = h2;
    d.HCAP = (uint32_t)c2;
  }
  if (gr) {  // receipt rings: twice the entries, every held entry moved to its position's new index
    const uint64_t b2 = 2ull * d.BCAP;
    if (N * b2 * 4 <= budget) {
      budget -= N * b2 * 4;
      uint32_t* rg2 = nullptr;
      if ((rc = dalloc(h, &rg2, N * b2))) return rc;
      launch_ring_move(d.rg, rg2, d.rhead, d.rtail, d.N, d.BCAP, (uint32_t)b2, st);
      HIPCK(hipStreamSynchronize(st));
      dfree(h, d.rg, 4ull * N * d.BCAP);
      d.rg = rg2;
      d.BCAP = (uint32_t)b2;
    }
  }
  if (gs) {  // slot table: twice the slots (whole 64-slot groups), or what the free HBM holds
    const uint64_t per = 2 * N + N / 4 + 64;  // S + HB + WB per slot, plus the slot arrays
    uint64_t s2 = std::min<uint64_t>(2ull * d.SPR, std::min<uint64_t>(1ull << 22, budget / per)) & ~63ull;
    if (s2 > d.SPR) {
      const uint64_t s1 = d.SPR, q1 = d.QW, q2 = s2 / 64;
      uint16_t* S2 = nullptr;
      unsigned long long *HB2 = nullptr, *WB2 = nullptr, *GU2 = nullptr, *DM2 = nullptr, *RX2 = nullptr;
      uint64_t *gid2 = nullptr, *key2 = nullptr;
      uint32_t *subj2 = nullptr, *ct2 = nullptr, *exp2 = nullptr, *used2 = nullptr, *fl2 = nullptr, *fexp2 = nullptr,
               *ag2 = nullptr, *rxl2 = nullptr;
      if ((rc = dalloc(h, &S2, N * s2)) || (rc = dalloc(h, &HB2, N * q2)) || (rc = dalloc(h, &WB2, N * q2)) ||
          (rc = dalloc(h, &GU2, q2)) || (rc = dalloc(h, &DM2, q2)) || (rc = dalloc(h, &ag2, q2)) ||
          (rc = dalloc(h, &gid2, s2)) || (rc = dalloc(h, &key2, s2)) || (rc = dalloc(h, &subj2, s2)) ||
          (rc = dalloc(h, &ct2, s2)) || (rc = dalloc(h, &exp2, s2)) || (rc = dalloc(h, &used2, s2)) ||
          (rc = dalloc(h, &fl2, s2)) || (rc = dalloc(h, &fexp2, s2))) {
        dfree(h, S2, 2 * N * s2), dfree(h, HB2, 8 * N * q2), dfree(h, WB2, 8 * N * q2), dfree(h, GU2, 8 * q2);
        dfree(h, DM2, 8 * q2), dfree(h, ag2, 4 * q2), dfree(h, gid2, 8 * s2), dfree(h, key2, 8 * s2);
        dfree(h, subj2, 4 * s2), dfree(h, ct2, 4 * s2), dfree(h, exp2, 4 * s2), dfree(h, used2, 4 * s2);
        dfree(h, fl2, 4 * s2);
        return rc;  // the old table stays in use
      }
      // rows: the old columns, then zero (no holder of a new slot)
      HIPCK(hipMemcpy2DAsync(S2, 2 * s2, d.S, 2 * s1, 2 * s1, N, hipMemcpyDeviceToDevice, st));
      HIPCK(hipMemset2DAsync(S2 + s1, 2 * s2, 0, 2 * (s2 - s1), N, st));
      HIPCK(hipMemcpy2DAsync(HB2, 8 * q2, d.HB, 8 * q1, 8 * q1, N, hipMemcpyDeviceToDevice, st));
      HIPCK(hipMemset2DAsync(HB2 + q1, 8 * q2, 0, 8 * (q2 - q1), N, st));
      HIPCK(hipMemcpy2DAsync(WB2, 8 * q2, d.WB, 8 * q1, 8 * q1, N, hipMemcpyDeviceToDevice, st));
      HIPCK(hipMemset2DAsync(WB2 + q1, 8 * q2, 0, 8 * (q2 - q1), N, st));
      HIPCK(hipMemsetAsync(GU2, 0, 8 * q2, st));
      HIPCK(hipMemsetAsync(DM2, 0, 8 * q2, st));
      HIPCK(hipMemcpyAsync(GU2, d.GU, 8 * q1, hipMemcpyDeviceToDevice, st));
      HIPCK(hipMemcpyAsync(DM2, d.DM, 8 * q1, hipMemcpyDeviceToDevice, st));
      HIPCK(hipMemcpyAsync(gid2, d.slot_gid, 8 * s1, hipMemcpyDeviceToDevice, st));
      HIPCK(hipMemcpyAsync(key2, d.slot_key, 8 * s1, hipMemcpyDeviceToDevice, st));
      HIPCK(hipMemcpyAsync(subj2, d.slot_subj, 4 * s1, hipMemcpyDeviceToDevice, st));
      HIPCK(hipMemcpyAsync(ct2, d.slot_ctick, 4 * s1, hipMemcpyDeviceToDevice, st));
      HIPCK(hipMemsetAsync(exp2, 0xFF, 4 * s2, st));  // new slots: unused, no expiry
      HIPCK(hipMemcpyAsync(exp2, d.slot_exp, 4 * s1, hipMemcpyDeviceToDevice, st));
      HIPCK(hipMemsetAsync(used2, 0, 4 * s2, st));
      HIPCK(hipMemcpyAsync(used2, d.slot_used, 4 * s1, hipMemcpyDeviceToDevice, st));
      // free list: the new ids below the old free entries (the old ones are taken first; ids are not observable)
      int32_t top = 0;
      HIPCK(hipMemcpyAsync(&top, d.free_top, 4, hipMemcpyDeviceToHost, st));
      HIPCK(hipStreamSynchronize(st));
      std::vector<uint32_t> ids(s2 - s1);
      for (uint64_t i = 0; i < s2 - s1; ++i) ids[i] = (uint32_t)(s2 - 1 - i);
      HIPCK(hipMemcpyAsync(fl2, ids.data(), 4 * ids.size(), hipMemcpyHostToDevice, st));
      if (top > 0) HIPCK(hipMemcpyAsync(fl2 + ids.size(), d.free_list, 4ull * top, hipMemcpyDeviceToDevice, st));
      const int32_t top2 = top + (int32_t)ids.size();
      HIPCK(hipMemcpyAsync(d.free_top, &top2, 4, hipMemcpyHostToDevice, st));
      // the per-tick contact rows follow the row width
      const uint32_t crcap = (uint32_t)std::max<uint64_t>(64, std::min<uint64_t>(4096, (512ull << 20) / (8ull * q2)));
      const uint32_t cr = getenv("SWIM_CAPS") && strstr(getenv("SWIM_CAPS"), "rx=") ? d.CRCAP : crcap;
      if ((rc = dalloc(h, &RX2, (uint64_t)cr * q2)) || (rc = dalloc(h, &rxl2, 3ull * cr))) return rc;
      HIPCK(hipStreamSynchronize(st));
      dfree(h, d.S, 2 * N * s1), dfree(h, d.HB, 8 * N * q1), dfree(h, d.WB, 8 * N * q1), dfree(h, d.GU, 8 * q1);
      dfree(h, d.DM, 8 * q1), dfree(h, d.agroup, 4 * q1), dfree(h, d.slot_gid, 8 * s1), dfree(h, d.slot_key, 8 * s1);
      dfree(h, d.slot_subj, 4 * s1), dfree(h, d.slot_ctick, 4 * s1), dfree(h, d.slot_exp, 4 * s1);
      dfree(h, d.slot_used, 4 * s1), dfree(h, d.free_list, 4 * s1), dfree(h, d.fexp, 4 * s1);
      dfree(h, d.RX, 8ull * d.CRCAP * q1), dfree(h, d.rxl, 12ull * d.CRCAP);
      d.S = S2, d.HB = HB2, d.WB = WB2, d.GU = GU2, d.DM = DM2, d.agroup = ag2, d.slot_gid = gid2, d.slot_key = key2;
      d.slot_subj = subj2, d.slot_ctick = ct2, d.slot_exp = exp2, d.slot_used = used2, d.free_list = fl2, d.fexp = fexp2;
      d.RX = RX2, d.rxl = rxl2, d.CRCAP = cr;
      d.SPR = d.SLOTS = (uint32_t)s2;
      d.QW = (uint32_t)q2;
    }
  }
  if (h->bytes == bytes0 && h->growths == growths0) {  // nothing fitted
    h->grow_next = h->tick + SCRUB;
    return SWIM_OK;
  }
  HIPCK(h2d(st, (void*)d.self, &d, sizeof(Dev)));
  h->growths++;
  return SWIM_OK;
}

// Capacity growth on a row shard (W > 1), after a tick whose gossip plane ran: the receipt rings and the incarnation
// history hold the replicated holder state, indexed by absolute ring positions and (gid, member) tags, so each shard
// sizes them for itself. The largest ring fill (this shard's targets in k_gossip_apply, the peers' first receipts in
// k_unpack_b) and the history entries are read back here (the speculative sharded batches never run the gossip
// plane, so this costs a stream sync only on gossip ticks). Slot ids are global (owner = id / SPR) and the per-tick
// lists feed fixed-size exchange regions, so those keep the sizes the config gives them.
static int grow_caps_shard(swim_handle* h) {
  Dev& d = h->d;
  if (!d.rfill) return SWIM_OK;
  uint32_t v[2] = {0, 0};
  HIPCK(hipMemcpyAsync(&v[0], d.rfill, 4, hipMemcpyDeviceToHost, h->stream));
  HIPCK(hipMemcpyAsync(&v[1], d.hist_n, 4, hipMemcpyDeviceToHost, h->stream));
  HIPCK(hipMemsetAsync(d.rfill, 0, 4, h->stream));
  HIPCK(hipStreamSynchronize(h->stream));
  volatile uint32_t* f = h->hflag;
  f[0] = 0;  // slots: not grown on a shard
  f[2] = v[0];
  f[3] = f[4] = f[5] = 0;
  f[6] = v[1];
  return grow_caps(h);
}

// NetworkLinkSettings.evaluateDelay (:64-74) quantised to ticks (SEMANTICS.md §2): thresholds on the 32-bit delay draw
// x, the extra ticks are the number of thresholds x reaches. false: a delay of 256 ticks or more is reachable.
bool delay_table(uint32_t D, uint32_t T, std::vector<uint32_t>* out) {
  out->clear();
  if (D == 0) return true;
  for (uint32_t j = 1; j <= 256; ++j) {
    const double th = std::ceil((1.0 - std::exp(-(double)j * (double)T / (double)D)) * 4294967296.0);
    if (th > 4294967295.0) return true;
    if (j == 256) return false;
    out->push_back((uint32_t)th);
  }
  return true;
}

bool to_ticks(uint32_t ms, uint32_t tick, uint32_t* out) {
  if (tick == 0 || ms % tick) return false;
  *out = ms / tick;
  return true;
}

int check_err(swim_handle* h) {
  hipError_t e = hipStreamSynchronize(h->stream);
  if (e != hipSuccess) {
    h->err = std::string("device failure: ") + hipGetErrorString(e);
    return SWIM_EDEVICE;
  }
  for (size_t i = 0; i < h->guards.size(); ++i) {  // SWIM_GUARD
    std::vector<unsigned char> g(2 * GUARD);
    const auto& a = h->guards[i];
    if (hipMemcpy(g.data(), a.first, GUARD, hipMemcpyDeviceToHost) != hipSuccess ||
        hipMemcpy(g.data() + GUARD, a.first + GUARD + a.second, GUARD, hipMemcpyDeviceToHost) != hipSuccess)
      return SWIM_EDEVICE;
    for (size_t j = 0; j < 2 * GUARD; ++j)
      if (g[j] != 0x5A) {
        h->err = "guard of allocation #" + std::to_string(i) + " (" + std::to_string(a.second) + " B) overwritten at " +
                 (j < GUARD ? "-" + std::to_string(GUARD - j) : "+" + std::to_string(j - GUARD)) + " value " +
                 std::to_string(g[j]);
        fprintf(stderr, "%s\n", h->err.c_str());
        return SWIM_EDEVICE;
      }
  }
  uint32_t eb[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  if (hipMemcpy(eb, h->d.err, sizeof(eb), hipMemcpyDeviceToHost) != hipSuccess) return SWIM_EDEVICE;
  uint32_t bits = eb[0];
  if (bits) {
    char hex[160];
    snprintf(hex, sizeof hex, "%x [info %u %u %u %u %u %u %u]", bits, eb[1], eb[2], eb[3], eb[4], eb[5], eb[6], eb[7]);
    h->err = std::string("engine capacity/semantic error bits 0x") + hex +
             " (see engine.h E_* ; raise the matching capacity in swim_config)";
    return SWIM_ECAPACITY;
  }
  return SWIM_OK;
}

// Host -> device update of engine state between ticks: ordered on the engine stream, so the next tick's kernels see
// it (a plain hipMemcpy runs on the null stream, which a non-blocking stream does not wait for), and finished before
// returning (the source is often a stack or vector buffer)
hipError_t h2d(hipStream_t st, void* dst, const void* src, size_t bytes) {
  hipError_t e = hipMemcpyAsync(dst, src, bytes, hipMemcpyHostToDevice, st);
  return e != hipSuccess ? e : hipStreamSynchronize(st);
}

// open a new NetworkEmulator-settings epoch that starts at the next tick to run
int push_epoch(swim_handle* h) {
  int e = h->cur_ep;
  if (h->ep_from[e] != (uint32_t)h->tick) e = (e + 1) % (int)MAX_EPOCHS;
  h->cur_ep = e;
  h->ep_from[e] = (uint32_t)h->tick;
  h->ep_loss[e] = h->loss;
  h->ep_part[e] = h->partitioned ? 1u : 0u;
  h->ep_delay[e] = h->delay_idx;
  // the kernels that take Dev by value see h->d at launch; the others read the device copy (d.self)
  Dev& d = h->d;
  d.ep_delay[e] = h->ep_delay[e];
  d.ep_from[e] = h->ep_from[e];
  d.ep_loss[e] = h->ep_loss[e];
  d.ep_part[e] = h->ep_part[e];
  HIPCK(h2d(h->stream, (void*)(d.self->ep_delay + e), &d.ep_delay[e], 4));
  HIPCK(h2d(h->stream, (void*)(d.self->ep_from + e), &d.ep_from[e], 4));
  HIPCK(h2d(h->stream, (void*)(d.self->ep_loss + e), &d.ep_loss[e], 4));
  HIPCK(h2d(h->stream, (void*)(d.self->ep_part + e), &d.ep_part[e], 4));
  HIPCK(h2d(h->stream, h->d.ep_group + (size_t)e * h->d.N, h->group.data(), 4ull * h->d.N));
  return SWIM_OK;
}

// rebuild the device link table from the host history (fault calls are rare; the table is at most ~300 KB)
int upload_links(swim_handle* h) {
  const uint32_t now = (uint32_t)h->tick, look = h->d.LOOKBACK + 2 * h->d.ping_t + 16;
  for (auto it = h->link_hist.begin(); it != h->link_hist.end();) {  // links back at default for long: forget them
    const auto& v = it->second;
    if (!h->link_cur.count(it->first) && v.back().second == LK_NONE && v.back().first + look < now)
      it = h->link_hist.erase(it);
    else
      ++it;
  }
  if (h->link_hist.size() > LKCAP / 2) {
    h->err = "more than 2048 links with custom NetworkEmulator settings";
    return SWIM_ECAPACITY;
  }
  std::vector<uint64_t> keys(LKCAP, 0);
  std::vector<uint32_t> hist((size_t)LKCAP * LKH * 2, LK_NONE);
  for (const auto& kv : h->link_hist) {
    uint32_t p = (uint32_t)mix64(kv.first) & (LKCAP - 1);
    while (keys[p]) p = (p + 1) & (LKCAP - 1);
    keys[p] = kv.first;
    const auto& v = kv.second;
    const size_t first = v.size() > LKH ? v.size() - LKH : 0;
    for (size_t i = first; i < v.size(); ++i) {
      hist[((size_t)p * LKH + (i - first)) * 2] = v[i].first;
      hist[((size_t)p * LKH + (i - first)) * 2 + 1] = v[i].second;
    }
    if (first) hist[(size_t)p * LKH * 2] |= LK_TRUNC;
  }
  uint32_t n = (uint32_t)h->link_hist.size();
  HIPCK(hipStreamSynchronize(h->stream));
  HIPCK(h2d(h->stream, h->d.link_key, keys.data(), 8ull * LKCAP));
  HIPCK(h2d(h->stream, h->d.link_hist, hist.data(), 4ull * hist.size()));
  h->d.link_n = n;
  HIPCK(h2d(h->stream, (void*)&h->d.self->link_n, &h->d.link_n, 4));
  return SWIM_OK;
}

// a change of link src -> dst effective from the next tick to run (NONE = back to the default settings)
void link_change(swim_handle* h, uint64_t key, uint32_t v) {
  auto& hv = h->link_hist[key];
  const uint32_t now = (uint32_t)h->tick;
  if (!hv.empty() && hv.back().first == now)
    hv.back().second = v;
  else
    hv.emplace_back(now, v);
  if (v == LK_NONE)
    h->link_cur.erase(key);
  else
    h->link_cur[key] = v;
}

uint64_t link_key_of(uint32_t src, uint32_t dst) { return (((uint64_t)src << 32) | dst) + 1ull; }

int build(swim_handle* h) {
  const swim_config& c = h->cfg;
  Dev& d = h->d;
  std::memset(&d, 0, sizeof(d));
  d.N = c.n_members;
  d.NS = (c.n_members + 7u) & ~7u;
  d.W = h->spec.world ? h->spec.world : 1u;
  d.rank = h->spec.rank;
  d.XW = 1;
  if (d.W > 1 && c.mode == SWIM_MODE_RUMOR) {  // slot sharding (engine.h): every shard runs every member
    d.XW = d.W;
    d.xrank = d.rank;
    d.W = 1;
    d.rank = 0;
  }
  d.lo = shard_lo(d.N, d.W, d.rank);
  d.hi = shard_lo(d.N, d.W, d.rank + 1);
  d.NL = d.hi - d.lo;
  d.F = c.gossip_fanout;
  d.kreq = c.ping_req_members;
  if (!to_ticks(c.ping_interval_ms, c.tick_ms, &d.ping_t) || !to_ticks(c.ping_timeout_ms, c.tick_ms, &d.pingTimeout_t) ||
      !to_ticks(c.gossip_interval_ms, c.tick_ms, &d.gossip_t) || !to_ticks(c.sync_interval_ms, c.tick_ms, &d.sync_t) ||
      !to_ticks(c.sync_timeout_ms, c.tick_ms, &d.syncTimeout_t) || !to_ticks(c.metadata_timeout_ms, c.tick_ms, &d.md_t) ||
      d.ping_t == 0 || d.gossip_t == 0 || d.sync_t == 0) {
    h->err = "every interval/timeout must be a positive multiple of tick_ms";
    return SWIM_EINVAL;
  }
  d.lat = c.latency_ticks;
  d.suspMult = c.suspicion_mult;
  d.repeatMult = c.gossip_repeat_mult;
  d.seed_lo = (uint32_t)c.seed;
  d.seed_hi = (uint32_t)(c.seed >> 32);
  d.init_mode = c.init_mode;
  d.mode = c.mode;
  d.n_dormant = c.n_dormant;
  d.churn = c.mode == SWIM_MODE_RUMOR ? c.churn_per_period : 0u;
  d.flags = c.flags;
  d.implicit = c.mode == SWIM_MODE_RUMOR && (c.n_members > 65536 || (c.flags & SWIM_FLAG_IMPLICIT_VIEWS)) ? 1u : 0u;
  d.fastp4 = c.mode == SWIM_MODE_RUMOR && !(c.flags & SWIM_FLAG_RECORD_EVENTS) ? 1u : 0u;
  d.exp = getenv("SWIM_EXP") ? (uint32_t)atoi(getenv("SWIM_EXP")) : 0u;  // timing experiments: wrong results
  // fast-structure capacities (include/swimhip_debug.h): SWIM_CAPS="trk=1,ulog=2,creq=1,cwmax=1,cev=1,mq=1,sort=2"
  // lowers them so that the exact fallbacks run; results stay bit-exact, only slower
  // undo log per member: a receiver merging thousands of records after a SYNC_ACK send (C2) would otherwise copy its
  // row on its own lane (cow_now); 1024 entries up to 65 536 members (8 KB each), 256 above
  d.ULOGC = c.n_members <= 65536 ? ULOG : 256;
  d.trk_cap = TRK, d.ulog_cap = d.ULOGC, d.creq_cap = CREQ, d.cwmax_cap = CWMAX, d.cev_cap = CEV, d.mq_cap = MQ;
  d.rr_atomic = getenv("SWIM_RR_ATOMIC") ? (uint32_t)atoi(getenv("SWIM_RR_ATOMIC")) : 64u;  // (measurements)
  d.hv = 24;  // routed receipts from which a member's P4 runs on a wave of its own (k_inbox_apply)
  d.XI = XINL;
  d.sort_cap = SORT_MAX;
  uint32_t rx_cap = NEVER, rp_cap = 0;
  const char* caps = getenv("SWIM_CAPS");
  if (caps) {
    std::string s(caps);
    size_t p = 0;
    while (p < s.size()) {
      size_t e = s.find(',', p);
      if (e == std::string::npos) e = s.size();
      const std::string kv = s.substr(p, e - p);
      p = e + 1;
      const size_t eq = kv.find('=');
      if (eq == std::string::npos) continue;
      const std::string k = kv.substr(0, eq);
      const uint32_t v = (uint32_t)strtoul(kv.c_str() + eq + 1, nullptr, 0);
      auto clampv = [&](uint32_t lo, uint32_t hi) { return std::max(lo, std::min(hi, v)); };
      if (k == "trk") d.trk_cap = clampv(0, TRK);
      else if (k == "ulog") d.ulog_cap = clampv(0, d.ULOGC);
      else if (k == "creq") d.creq_cap = clampv(1, CREQ);
      else if (k == "cwmax") d.cwmax_cap = clampv(0, CWMAX);
      else if (k == "cev") d.cev_cap = clampv(0, CEV);
      else if (k == "mq") d.mq_cap = clampv(1, MQ);
      else if (k == "hv") d.hv = std::max<uint32_t>(1, v);  // k_inbox_apply from this many receipts
      else if (k == "rx") rx_cap = v;
      else if (k == "rp") rp_cap = std::max<uint32_t>(64, v);  // replay / slow-path send lists (grow_caps tests)
      else if (k == "xinl") d.XI = std::max<uint32_t>(64, std::min<uint32_t>(XINL, v)) & ~7u;  // send/recv group past it
      else if (k == "sort") {
        uint32_t r = 2;
        while (r * 2 <= clampv(2, SORT_MAX)) r *= 2;  // a power of two (bitonic runs)
        d.sort_cap = r;
      }
    }
  }
  // seeds: LinkedHashSet of valid ids (MembershipProtocolImpl.java:160-166); self is skipped per member
  for (uint32_t i = 0; i < c.n_seeds; ++i) {
    uint32_t s = c.seeds[i];
    if (s >= d.N) continue;
    bool dup = false;
    for (uint32_t j = 0; j < d.n_seeds; ++j) dup |= d.seeds[j] == s;
    if (!dup) d.seeds[d.n_seeds++] = s;
  }
  const uint64_t N = d.N;
  // FD / gossip lists: a member can be listed twice when its REMOVED overtakes the metadata fetch of its ADDED
  // (emitMembershipEvent :543-588 is asynchronous), so the lists get slack beyond N - 1 entries
  d.LCAP = d.N + (c.list_slack ? c.list_slack : 64);
  d.FCAP = c.pending_fetch_cap ? c.pending_fetch_cap : 256;
  d.GRCAP = c.init_mode == SWIM_INIT_COLD_JOIN ? std::min<uint32_t>(d.N + 16, 1024) : 32;
  if (d.implicit) d.FCAP = d.GRCAP = 1;  // RUMOR mode: no metadata fetch, no SYNC reply group
  uint32_t maxSpread = d.repeatMult * (32u - (uint32_t)__builtin_clz(d.LCAP + 1));
  // link delays (swim_config.delay_cap_ms): the longest delay in ticks past lat
  {
    std::vector<uint32_t> t;
    if (!delay_table(c.delay_cap_ms, c.tick_ms, &t)) {
      h->err = "delay_cap_ms above 11 x tick_ms";
      return SWIM_EINVAL;
    }
    d.EMAX = (uint32_t)t.size();
    d.PCAP = c.delay_cap_ms ? PATHCAP_DELAY : PATHCAP;
  }
  d.LOGW = 8;
  // rounds kept for the infectedFrom replay (a delayed send arrives up to EMAX ticks after its round)
  while (d.LOGW < 4 * (maxSpread + 2) + 2 * ((d.EMAX + d.gossip_t - 1) / d.gossip_t + 1)) d.LOGW <<= 1;
  d.LOOKBACK = d.LOGW * d.gossip_t;
  d.gt_mul = d.gossip_t == 1 ? 0xFFFFFFFFu : (uint32_t)((1ull << 32) / d.gossip_t);
  // incarnation history of reborn (gossip, member) pairs (88 B per entry). 2^20 entries (92 MB) by default; a run
  // that asks for a large slot table (a storm: C4's heal rebirths a large share of the holder states) gets one
  // entry per 8 holder states, up to 2^24; SWIM_HIST_CAP overrides (a full table raises E_REBORN, info 1)
  {
    uint64_t hc = 1u << 20;
    if (c.gossip_slot_cap) {
      const uint64_t want = (uint64_t)c.gossip_slot_cap * N / 8;
      while (hc < want && hc < (1u << 24)) hc <<= 1;
    }
    if (const char* e = getenv("SWIM_HIST_CAP")) {
      hc = 1024;
      while (hc < strtoull(e, nullptr, 0) && hc < (1u << 26)) hc <<= 1;
    }
    d.HCAP = (uint32_t)hc;
  }
  // default: 64 slots per member, at most 32 GB of holder table (C2's SYNC re-spread storm keeps ~10^5 gossips alive)
  uint64_t slots = c.gossip_slot_cap ? c.gossip_slot_cap
                                     : std::min<uint64_t>(1ull << 22, std::max<uint64_t>(1024, std::min<uint64_t>(64 * N, (32ull << 30) / (4 * N))));
  // RUMOR mode with churn (C5): the rumors alive together follow from the config. A rumor reaches every member in
  // about 2 log2(N) rounds and its slot is recycled EXPB = 2 maxSpread + 4 rounds after its last receipt, so about
  // churn x (2 maxSpread + 4 + 2 bitlen(N)) gossip intervals' worth are alive, split over the XW slot shards (+10 %);
  // a member holds the ones of its last 2 maxSpread + 3 rounds (its receipt ring, below). Growth (grow_caps) covers
  // what this misses.
  uint64_t rumor_ring = 0;
  if (!c.gossip_slot_cap && c.mode == SWIM_MODE_RUMOR && c.churn_per_period) {
    const uint64_t life = (2ull * maxSpread + 4 + 2ull * bitlen(d.N)) * d.gossip_t;
    const uint64_t held = (2ull * maxSpread + 3) * d.gossip_t;
    slots = std::min<uint64_t>(1ull << 22, std::max<uint64_t>(1024, 11 * c.churn_per_period * life / (10 * d.ping_t * d.XW)));
    rumor_ring = 21 * c.churn_per_period * held / (20 * d.ping_t * d.XW);
  }
  // every shard allocates new gossips from its own slot range; the slot table itself is replicated, so the ranges
  // split the budget (twice over, for shards that create more than their share) instead of multiplying it by W: at
  // 100k members and W = 8 a full range per shard would be a 275 GB holder table on every GPU
  const uint64_t share = d.W == 1 ? slots : std::max<uint64_t>(1024, (2 * slots + d.W - 1) / d.W);
  d.SPR = (uint32_t)std::min<uint64_t>(std::min<uint64_t>(slots, share), (1ull << 22) / d.W);
  d.SPR = (d.SPR + 63u) & ~63u;  // whole 64-slot groups per shard (holder bit rows)
  d.SLOTS = d.SPR * d.W;
  d.QW = d.SLOTS / 64;
  // a gossip's holders have all swept it within 2 (spread + 1) + 2 of their rounds after their receipt
  // (sweepGossips :283-308, spread <= maxSpread): its slot is recycled after that (slot_exp)
  d.EXPB = (2u * maxSpread + 4u) * d.gossip_t;
  if (2u * maxSpread + 4u >= 500u) {  // receipt-ring entries keep the infection period modulo 1024 (gossip.hip)
    h->err = "gossipRepeatMult x ceilLog2(members) too large (at most 248)";
    return SWIM_EINVAL;
  }
  // 16-bit holder entries (engine.h S16_*): a gossip slot may stay in use SLIFE ticks. Its holders sweep it EXPB
  // ticks after their receipt, and an epidemic's first receipts come within about maxSpread + 1 rounds of its
  // creation, so a slot lives about (3 maxSpread + 6) gossip intervals. A config whose gossip interval is so many
  // ticks that this reaches SLIFE is refused here instead of failing with E_SLIFE mid-run
  if ((3ull * maxSpread + 6ull) * d.gossip_t >= SLIFE) {
    h->err = "gossipInterval / tick_ms x (3 x gossipRepeatMult x ceilLog2(members) + 6) must stay below " +
             std::to_string(SLIFE) + " ticks (the holder entries' tick window): use a coarser tick_ms";
    return SWIM_EINVAL;
  }
  // receipt ring per member: at least as many entries as the member can hold gossips; by default the slot table's
  // size, within about 16-24 GB in all (C2 holds ~3·10^5 gossips per member at 10k members), and
  // swim_config.gossip_ring_cap overrides (a full ring raises E_RING)
  {
    const uint64_t want = c.gossip_ring_cap ? c.gossip_ring_cap : rumor_ring ? std::max<uint64_t>(4096, rumor_ring)
                                            : std::min<uint64_t>(d.SLOTS, std::max<uint64_t>(4096, (16ull << 30) / (4 * N)));
    uint64_t bc = 64;
    while (bc < want && bc < (1ull << 31)) bc <<= 1;
    if (!c.gossip_ring_cap && !rumor_ring && bc > 4096 && bc * N * 4 > (24ull << 30)) bc >>= 1;
    d.BCAP = (uint32_t)bc;
  }
  uint64_t mc = N / d.sync_t * 4 + N / d.ping_t + 1024;
  if (c.init_mode == SWIM_INIT_COLD_JOIN) mc = std::max<uint64_t>(mc, N + 1024);
  d.MSGCAP = (uint32_t)mc;
  d.NCHUNK = (uint32_t)((d.NS + CH - 1) / CH);
  d.NMETA = (uint32_t)((d.NS + MCH - 1) / MCH);
  d.POOLCAP = (uint32_t)std::min<uint64_t>(1ull << 26, std::max<uint64_t>(1ull << 20, N * 64));
  d.EVCAP = c.event_cap ? c.event_cap : (1u << 20);
  // first receipts per tick: routed to P4 (RCAP), shipped to the other row shards (DCAP)
  d.DCAP = (uint32_t)std::min<uint64_t>(1ull << 27, std::max<uint64_t>(1ull << 16, N * 16384));
  d.RCAP = d.DCAP;
  // infectedFrom replays: in a small cluster most pairs have a logged contact, so under a DEAD-gossip storm nearly
  // every send is replayed (C4 at 2 000 members: ~4·10^7 per tick)
  d.SLOWCAP = d.RPCAP = std::max<uint32_t>(d.DCAP, 1u << 26);
  if (const char* dc = getenv("SWIM_DELIV_CAP")) {  // experiments (tools/exp_c4.py): first receipts per tick
    d.DCAP = d.RCAP = (uint32_t)std::min<uint64_t>(1ull << 30, strtoull(dc, nullptr, 0));
    d.SLOWCAP = d.RPCAP = std::max(d.SLOWCAP, d.DCAP);
  }
  if (rp_cap) d.SLOWCAP = d.RPCAP = rp_cap;
  if (d.implicit) {
    // C5: every period's rumors start at one tick, so their epidemics peak together: on one of 8 slot shards a tick
    // can deliver ~7·10^8 first receipts (8 B each). Their GOSSIP events skip the receipt routing (fastp4), and
    // infectedFrom replays are rare at this size.
    d.DCAP = 1u << 30;
    d.RCAP = d.fastp4 ? 1u << 22 : 1u << 28;
    d.SLOWCAP = d.RPCAP = 1u << 26;
  }
  // copy-on-write snapshots and pinned payload copies (pin_msg) per tick: up to 256 MB per buffer, at least 64 rows
  d.ARENA_ROWS = (uint32_t)std::min<uint64_t>(d.MSGCAP, std::max<uint64_t>(64, (256ull << 20) / (4ull * d.NS)));
  if (d.implicit) {  // no SYNC traffic: minimal message buffers
    d.MSGCAP = 1024;
    d.ARENA_ROWS = 1;
    d.POOLCAP = 1024;
  }

  int rc;
#define A(p, n)                                   \
  if ((rc = dalloc(h, &(p), (size_t)(n))) != 0) return rc;
  A(d.link_key, LKCAP) A(d.link_hist, (uint64_t)LKCAP * LKH * 2)
  A(d.dead_tick, N)
  A(d.dly_thr, DTAB * 256) A(d.dly_len, DTAB)
  A(d.ep_group, MAX_EPOCHS * N) A(d.md_version, N)
  A(d.nextPing, N) A(d.nextGossip, N) A(d.nextSync, N) A(d.held, N) A(d.timerMin, N) A(d.initFlags, N)
  A(d.firstGossip, N) A(d.ms, N) A(d.sel, N * 8)
  const uint64_t NL = d.NL;  // per-observer arrays: this shard's rows only
  const uint64_t NV = d.implicit ? 1 : NL;  // implicit views: no table or list is stored
  A(d.rowk, NV * d.NS) A(d.rowa, NV * d.NS) A(d.fdl, NV * d.LCAP) A(d.gl, NV * d.LCAP)
  d.rowk8 = nullptr;  // allocated last, if it fits (below)
  d.base_row8 = nullptr;
  d.NS8 = (c.n_members + 15u) & ~15u;
  A(d.subs, NL * SUBCAP * 4) A(d.paths, NL * d.PCAP * 5) A(d.fetch, NL * d.FCAP * FREC) A(d.groups, NL * d.GRCAP * GREC)
  A(d.tround, N) A(d.tcnt, N) A(d.tspread, N) A(d.tperiod, N) A(d.T, N * d.F) A(d.tcontact, N * d.F) A(d.slow, d.SLOWCAP) A(d.slow_n, 1) A(d.rp, d.RPCAP) A(d.rp_n, 1) A(d.start_tick, N) A(d.jseed_n, N) A(d.jseeds, 16 * N) A(d.md_uidx, N) A(d.mcfg, 4 * N) A(d.md_ver, NL * MDU) A(d.churn_q, 2ull * d.churn) A(d.ucnt, N) A(d.cin, N * d.F) A(d.HB, (uint64_t)d.QW * N) A(d.WB, (uint64_t)d.QW * N) A(d.cev, N * d.F * CEVW)
  A(d.rg, (uint64_t)d.BCAP * N) A(d.rhead, N) A(d.rwin, N) A(d.rseen, N) A(d.rtail, N) A(d.rwl, N) A(d.nrwl, 1)
  A(d.rsend, N) A(d.rwnew, N) A(d.GU, d.QW) A(d.DM, d.QW) A(d.agroup, d.QW) A(d.nagroup, 2)
  A(d.tin_cnt, N) A(d.tin_off, N) A(d.tin_fill, N) A(d.tin, N * d.F) A(d.tlist, N) A(d.ntl, 1) A(d.rt0, N)
  d.CRCAP = (uint32_t)std::max<uint64_t>(64, std::min<uint64_t>(4096, (512ull << 20) / (8ull * d.QW)));
  if (rx_cap != NEVER) d.CRCAP = rx_cap;  // SWIM_CAPS rx=...: contact pairs past it replay their whole window
  A(d.crow, N * d.F) A(d.RX, (uint64_t)d.CRCAP * d.QW) A(d.rxl, 3ull * d.CRCAP) A(d.nrx, 1) A(d.cfl, N * d.F) A(d.ncfl, 1)
  A(d.log_tick, N * d.LOGW) A(d.log_spread, N * d.LOGW) A(d.log_cnt, N * d.LOGW) A(d.log_tg, N * d.LOGW * d.F)
  A(d.log_pos, N) A(d.spchg, N)
  A(d.slot_gid, d.SLOTS) A(d.slot_subj, d.SLOTS) A(d.slot_ctick, d.SLOTS) A(d.slot_key, d.SLOTS) A(d.slot_exp, d.SLOTS)
  A(d.slot_used, d.SLOTS) A(d.S, (uint64_t)d.SLOTS * N) A(d.free_list, d.SLOTS) A(d.free_top, 1)
  A(d.xd, d.W > 1 ? d.DCAP : 1) A(d.xd_n, 1) A(d.rc_raw, d.RCAP) A(d.rc_n, 1) A(d.rc_cnt, N) A(d.rc_off, N) A(d.rc_fill, N) A(d.scan_part, 1024)
  A(d.rc_slot, d.RCAP) A(d.rc_ndrop, N) A(d.dead_rx, N) A(d.leaving, N) A(d.rc_key, d.RCAP) A(d.rc_slot2, d.RCAP) A(d.rc_key2, d.RCAP) A(d.fexp, d.SLOTS) A(d.nfexp, 1) A(d.hist, (uint64_t)d.HCAP * HREC)
  A(d.msgs[0], d.MSGCAP) A(d.msgs[1], d.MSGCAP) A(d.nmsg, 2) A(d.arena[0], (uint64_t)d.ARENA_ROWS * d.NS)
  A(d.arena[1], (uint64_t)d.ARENA_ROWS * d.NS) A(d.arena_used, 2)
  A(d.m_next, 2ull * d.MSGCAP) A(d.m_head, 2 * N) A(d.next_evt, N) A(d.mdone, 2) A(d.trk, NL * TRKL) A(d.ulog, NL * d.ULOGC * 2) A(d.spq, NL * SPQ * 8) A(d.fpend, NL * KP * 2) A(d.pending_inc, N) A(d.chunk_meta, (uint64_t)d.MSGCAP * d.NMETA * 2)
  A(d.pool, d.POOLCAP) A(d.pool_used, 1)
  d.NW = d.implicit ? 0u : (d.N + 63u) / 64u;  // (RUMOR mode with implicit views has no SYNC)
  A(d.hv_list, NL) A(d.nhv, 1) A(d.hv_pend, NL) A(d.hv_tlast, NL) A(d.sg_list, N) A(d.nsg, 1) A(d.ap_list, N) A(d.nap, 1)
  HIPCK(hipMemsetAsync(d.nhv, 0, 4, h->stream));
  A(d.tbm, std::max<uint64_t>(1, NL * d.NW))
  HIPCK(hipMemsetAsync(d.tbm, 0, 8 * std::max<uint64_t>(1, NL * d.NW), h->stream));
  // SYNC_ACK resolution (k_ack_resolve); SWIM_NO_ACKRES streams every payload (measurements)
  d.ackres = !d.implicit && !getenv("SWIM_NO_ACKRES") ? 1u : 0u;
  if (d.ackres) {
    A(d.tlog, 2 * NL * TL) A(d.tl_n, 2 * NL) A(d.tl_tick, 2 * NL) A(d.dlist, 4ull * d.MSGCAP) A(d.ndl, 1) A(d.dlist_w, 4ull * d.MSGCAP) A(d.ndlw, 1)
    if (d.W > 1) A(d.mlog, (uint64_t)d.MSGCAP * TL)
    HIPCK(hipMemsetAsync(d.tl_tick, 0xFF, 8 * NL, h->stream));
    HIPCK(hipMemsetAsync(d.ndl, 0, 4, h->stream));
    HIPCK(hipMemsetAsync(d.ndlw, 0, 4, h->stream));
  }
  // capacity growth between ticks (grow_caps), without guard zones; SWIM_NO_GROW keeps the sizes fixed. A row shard
  // grows its receipt rings and incarnation history (grow_caps_shard); its slot ids and exchange capacities are global
  if (!getenv("SWIM_NO_GROW") && !getenv("SWIM_GUARD")) {
    A(d.rfill, 1) A(d.hist_n, 1)
    HIPCK(hipMemsetAsync(d.rfill, 0, 4, h->stream));
    HIPCK(hipMemsetAsync(d.hist_n, 0, 4, h->stream));
  }
  A(d.ev, (uint64_t)d.EVCAP * 8) A(d.ev_n, 1) A(d.ctr, C_NCTR) A(d.ctr_sh, (uint64_t)CSH * CSTRIDE) A(d.err, 8)
  if (c.flags & SWIM_FLAG_EMULATOR_COUNTERS) {
    A(d.em, 2 * N)
    HIPCK(hipMemsetAsync(d.em, 0, 16 * N, h->stream));
  }
  if (d.EMAX) {  // delayed gossip receipts by delivery tick; delayed SYNC / SYNC_ACK messages with their payloads
    d.DQCAP = (uint32_t)std::min<uint64_t>(1ull << 22, std::max<uint64_t>(1ull << 16, (1ull << 30) / (8ull * (d.EMAX + 2))));
    A(d.dq, (uint64_t)(d.EMAX + 2) * d.DQCAP) A(d.dq_n, d.EMAX + 2) A(d.dmark, N)
    HIPCK(hipMemsetAsync(d.dq_n, 0, 4ull * (d.EMAX + 2), h->stream));
    HIPCK(hipMemsetAsync(d.dmark, 0, 4 * N, h->stream));
    d.DSCAP = (uint32_t)std::max<uint64_t>(64, std::min<uint64_t>(4096, (256ull << 20) / (4ull * d.NS)));
    A(d.ds_msg, d.DSCAP) A(d.ds_row, (uint64_t)d.DSCAP * d.NS) A(d.ds_used, d.DSCAP) A(d.ds_free, d.DSCAP) A(d.ds_top, 1)
    HIPCK(hipMemsetAsync(d.ds_used, 0, 4ull * d.DSCAP, h->stream));
    std::vector<uint32_t> fl(d.DSCAP);
    for (uint32_t i = 0; i < d.DSCAP; ++i) fl[i] = i;
    const int32_t top = (int32_t)d.DSCAP;
    HIPCK(h2d(h->stream, d.ds_free, fl.data(), 4ull * d.DSCAP));
    HIPCK(h2d(h->stream, d.ds_top, &top, 4));
  }
  if (d.exp & 512) A(d.wt, (uint64_t)(NL + 255) / 256 * 4 * 16)
  if (d.fastp4) {
    A(d.evp_hash, N) A(d.evp_n, N)
    HIPCK(hipMemsetAsync(d.evp_hash, 0, 8 * N, h->stream));
    HIPCK(hipMemsetAsync(d.evp_n, 0, 4 * N, h->stream));
  }
  if (d.XW > 1) {
    A(d.held_delta, N)
    HIPCK(hipMemsetAsync(d.held_delta, 0, 4 * N, h->stream));
    if (h->spec.transport == SWIM_TRANSPORT_HOST) {
      h->hsend.resize(4ull * N * d.XW);
      h->hrecv.resize(4ull * N * d.XW);
    }
  }
  if (getenv("SWIM_CAPS") || getenv("SWIM_FALLBACKS")) {  // count the capacity fallbacks (swim_debug_fallbacks)
    A(d.fb, FB_N)
    HIPCK(hipMemsetAsync(d.fb, 0, 8 * FB_N, h->stream));
  }
  if (getenv("SWIM_SEND_LOG")) {  // debugging aid: every counted gossip send
    d.dbg_send_cap = (uint32_t)atoi(getenv("SWIM_SEND_LOG"));
    A(d.dbg_send, 5ull * d.dbg_send_cap) A(d.dbg_send_n, 1)
    HIPCK(hipMemsetAsync(d.dbg_send_n, 0, 4, h->stream));
  }
  if (d.W > 1) {
    d.MW = (d.NCHUNK + 63) / 64;
    d.NSCAP = 1u << 16;
    d.RRCAP = d.NL;
    d.RQCAP = d.MSGCAP;
    d.RXCAP = d.MSGCAP;
    d.CHCAP = h->spec.chunk_cap ? h->spec.chunk_cap : (uint32_t)std::min<uint64_t>(4096, (uint64_t)d.MSGCAP * d.NCHUNK);
    uint64_t se = sync_entry_size(d.MW);
    d.XA_PEER = ((32 + 4ull * NSW * d.NSCAP + 4ull * RRW * d.RRCAP + se * d.RQCAP + 511) & ~255ull) +
                (uint64_t)d.CHCAP * CH * 4;
    d.XB_PEER = 16 + 8ull * std::min<uint64_t>((uint64_t)d.DCAP, 1ull << 25);
    A(d.rdirty, (uint64_t)NL * d.MW) A(d.arena_dirty[0], (uint64_t)d.ARENA_ROWS * d.MW)
    A(d.arena_dirty[1], (uint64_t)d.ARENA_ROWS * d.MW)
    A(d.base_row, d.NS) A(d.xn, 8) A(d.ns_rec, (uint64_t)d.NSCAP * NSW) A(d.rr_rec, (uint64_t)d.RRCAP * RRW)
    A(d.mtmp, d.MSGCAP) A(d.rx_mask, (uint64_t)d.RXCAP * d.MW) A(d.rx_off, d.RXCAP)
    A(d.xa_send, d.W * d.XA_PEER) A(d.xa_recv, d.W * d.XA_PEER) A(d.xb_send, d.W * d.XB_PEER)
    A(d.xb_recv, d.W * d.XB_PEER) A(d.xa_scnt, d.W) A(d.xa_rcnt, d.W) A(d.xb_scnt, d.W) A(d.xb_rcnt, d.W)
    HIPCK(hipMemsetAsync(d.xa_rcnt, 0, 8ull * d.W, h->stream));
    HIPCK(hipMemsetAsync(d.xb_rcnt, 0, 8ull * d.W, h->stream));
    HIPCK(hipHostMalloc((void**)&h->hcnt, 16ull * d.W, hipHostMallocDefault));
    A(d.xi_send, (uint64_t)d.W * XINL) A(d.xi_recv, (uint64_t)d.W * XINL)
    A(d.xdone, 2ull * d.W)  // [0]: peer columns done (k_pack_all), [1 + q]: blocks of column q done
    HIPCK(hipMemsetAsync(d.xdone, 0, 8ull * d.W, h->stream));
    d.inl = h->spec.transport == SWIM_TRANSPORT_RCCL ? 1u : 0u;
    HIPCK(hipHostMalloc((void**)&h->xi_host_h, 16ull * d.W, hipHostMallocMapped | hipHostMallocCoherent));
    HIPCK(hipHostGetDevicePointer((void**)&d.xi_host, (void*)h->xi_host_h, 0));
    if (h->spec.transport == SWIM_TRANSPORT_HOST) {
      h->hsend.resize(d.W * std::max(d.XA_PEER, d.XB_PEER));
      h->hrecv.resize(d.W * std::max(d.XA_PEER, d.XB_PEER));
    }
  }
  // stored tables: the diff's 8-bit shadow plane of this shard's rows, only when it fits beside everything else with
  // the usual growth reserve (an optimisation: without it k_sync_diff and row_put use the u32 keys; SWIM_NO_K8 forces
  // that). On a row shard it serves the payloads of local senders; peers' payloads arrive as u32 chunks
  if (!d.implicit && !getenv("SWIM_NO_K8")) {
    size_t fr = 0, tot = 0;
    HIPCK(hipMemGetInfo(&fr, &tot));
    if ((uint64_t)fr > NV * d.NS8 + (4ull << 30)) {
      A(d.rowk8, NV * d.NS8)
      if (d.W > 1) A(d.base_row8, d.NS8)
    }
  }
#undef A
  HIPCK(hipMemsetAsync(d.S, 0, (size_t)d.SLOTS * N * 2, h->stream));
  HIPCK(hipMemsetAsync(d.HB, 0, (size_t)d.QW * N * 8, h->stream));
  HIPCK(hipMemsetAsync(d.WB, 0, (size_t)d.QW * N * 8, h->stream));
  HIPCK(hipMemsetAsync(d.GU, 0, (size_t)d.QW * 8, h->stream));
  HIPCK(hipMemsetAsync(d.DM, 0, (size_t)d.QW * 8, h->stream));
  HIPCK(hipMemsetAsync(d.nagroup, 0, 8, h->stream));
  HIPCK(hipMemsetAsync(d.ctr, 0, C_NCTR * 8, h->stream));
  HIPCK(hipMemsetAsync(d.ctr_sh, 0, 8ull * CSH * CSTRIDE, h->stream));
  HIPCK(hipMemsetAsync(d.hist, 0, (size_t)d.HCAP * HREC * 8, h->stream));
  HIPCK(hipMemsetAsync(d.err, 0, 32, h->stream));
  HIPCK(hipMemsetAsync(d.ev_n, 0, 4, h->stream));
  HIPCK(hipMemsetAsync(d.nmsg, 0, 8, h->stream));
  HIPCK(hipMemsetAsync(d.arena_used, 0, 8, h->stream));
  HIPCK(hipMemsetAsync(d.tcnt, 0, N * 4, h->stream));
  HIPCK(hipMemsetAsync(d.ucnt, 0, N * 4, h->stream));
  HIPCK(hipMemsetAsync(d.pool_used, 0, 4, h->stream));
  HIPCK(hipMemsetAsync(d.mdone, 0, 8, h->stream));
  d.halt = d.mdone + 1;
  d.link_n = 0;
  HIPCK(hipMemsetAsync(d.link_key, 0, 8ull * LKCAP, h->stream));
  HIPCK(hipMemsetAsync(d.xd_n, 0, 4, h->stream));
  HIPCK(hipMemsetAsync(d.rc_n, 0, 4, h->stream));
  HIPCK(hipMemsetAsync(d.rc_ndrop, 0, 4 * N, h->stream));
  HIPCK(hipMemsetAsync(d.dead_rx, 0, 4 * N, h->stream));
  HIPCK(hipMemsetAsync(d.leaving, 0, 4 * N, h->stream));
  HIPCK(hipMemsetAsync(d.m_head, 0xFF, 2 * N * 4, h->stream));
  HIPCK(hipMemsetAsync(d.msgs[0], 0xFF, (size_t)d.MSGCAP * sizeof(SyncMsg), h->stream));  // pin = NEVER (send_sync)
  HIPCK(hipMemsetAsync(d.msgs[1], 0xFF, (size_t)d.MSGCAP * sizeof(SyncMsg), h->stream));
  if (d.W > 1) {
    HIPCK(hipMemsetAsync(d.xn, 0, 32, h->stream));
    HIPCK(hipMemsetAsync(d.xa_scnt, 0, 8ull * d.W, h->stream));
    HIPCK(hipMemsetAsync(d.xb_scnt, 0, 8ull * d.W, h->stream));
  }
  HIPCK(hipHostMalloc((void**)&h->hflag, 64, hipHostMallocMapped | hipHostMallocCoherent));
  for (int i = 0; i < 16; ++i) h->hflag[i] = 0;
  HIPCK(hipHostGetDevicePointer((void**)&d.hflag, (void*)h->hflag, 0));
  if ((rc = dalloc(h, &d.hsh, 8)) != 0) return rc;
  HIPCK(hipMemsetAsync(d.hsh, 0, 32, h->stream));  // (hflag above: all zero)
  HIPCK(hipEventCreateWithFlags(&h->ev_member, hipEventDisableTiming));
  HIPCK(hipMemsetAsync(d.subs, 0, NL * SUBCAP * 16, h->stream));
  int32_t top = (int32_t)d.SPR;
  HIPCK(hipMemcpyAsync(d.free_top, &top, 4, hipMemcpyHostToDevice, h->stream));
  {  // every member starts with the swim_config FailureDetectorConfig and sync group 0 (swim_set_member_config)
    std::vector<uint32_t> mc(4ull * N);
    for (uint64_t m = 0; m < N; ++m) {
      mc[4 * m] = d.ping_t;
      mc[4 * m + 1] = d.pingTimeout_t;
      mc[4 * m + 2] = d.kreq;
      mc[4 * m + 3] = 0;
    }
    HIPCK(hipMemcpyAsync(d.mcfg, mc.data(), 16ull * N, hipMemcpyHostToDevice, h->stream));
    HIPCK(hipStreamSynchronize(h->stream));
  }
  for (uint32_t e = 0; e < MAX_EPOCHS; ++e) d.ep_from[e] = NEVER;  // (uploaded with Dev below)
  HIPCK(hipStreamSynchronize(h->stream));  // `top` lives on this stack frame
  h->group.assign(d.N, 0);
  for (uint32_t e = 0; e < MAX_EPOCHS; ++e) h->ep_from[e] = NEVER;
  h->cur_ep = 0;
  // every initialisation above is ordered on the engine stream (a non-blocking stream does not wait for the
  // legacy null stream, so a plain hipMemset could still be running when the first tick starts)
  Dev* dcopy = nullptr;
  if ((rc = dalloc(h, &dcopy, 1)) != 0) return rc;
  d.self = dcopy;
  HIPCK(hipMemcpyAsync(dcopy, &d, sizeof(Dev), hipMemcpyHostToDevice, h->stream));
  HIPCK(hipStreamSynchronize(h->stream));
  launch_init(d, h->stream);
  if ((rc = push_epoch(h)) != 0) return rc;
  return check_err(h);
}

// The host waits for the end of every tick's exchange A. A blocking event wait falls back to an interrupt after a
// short active phase, and that wake-up would stall the GPU, which has nothing queued behind the exchange: spin.
hipError_t spin_wait(hipEvent_t ev) {
  hipError_t e;
  while ((e = hipEventQuery(ev)) == hipErrorNotReady) {
  }
  return e;
}

// RCCL, fixed-size part of an exchange: the inline all-to-all and its unpacking into the regions (k_inline_in also
// publishes the count words to the host-mapped xi_host)
int exchange_inline(swim_handle* h, uint8_t* recv, uint64_t cap, unsigned long long* scnt, unsigned long long* rcnt,
                    bool spec) {
  if (ncclAllToAll(h->d.xi_send, h->d.xi_recv, h->d.XI, ncclUint8, h->comm, h->stream) != ncclSuccess) {
    h->err = "ncclAllToAll (inline exchange) failed";
    return SWIM_EDEVICE;
  }
  launch_inline_in(h->d, recv, cap, scnt, rcnt, h->stream, spec);
  return SWIM_OK;
}

// RCCL, after the inline part has completed: the count words from xi_host (the gossip flag, the sizes) and a
// send/recv group for the regions that did not fit inline
int exchange_rest(swim_handle* h, uint8_t* send, uint8_t* recv, uint64_t cap) {
  const uint32_t W = h->d.W, me = h->d.rank;
  unsigned long long* hc = h->hcnt;
  volatile unsigned long long* xh = h->d.xi_host;
  for (uint32_t q = 0; q < 2 * W; ++q) hc[q] = xh[q];
  h->xflag = false;
  bool rest = false;
  for (uint32_t q = 0; q < 2 * W; ++q) {
    h->xflag |= (hc[q] & XFLAG_GOSSIP) != 0;
    rest |= (hc[q] & XCNT_MASK) > h->d.XI - 8;
    if ((hc[q] & XCNT_MASK) > cap) {
      h->err = "exchange block larger than its region";
      return SWIM_ECAPACITY;
    }
  }
  if (rest) {
    bool ok = ncclGroupStart() == ncclSuccess;
    for (uint32_t q = 0; q < W && ok; ++q) {
      if (q == me) continue;
      const uint64_t sb = hc[q] & XCNT_MASK, rb = hc[W + q] & XCNT_MASK;
      const uint64_t X = h->d.XI - 8;
      if (sb > X) ok &= ncclSend(send + (size_t)q * cap + X, sb - X, ncclUint8, (int)q, h->comm, h->stream) == ncclSuccess;
      if (rb > X) ok &= ncclRecv(recv + (size_t)q * cap + X, rb - X, ncclUint8, (int)q, h->comm, h->stream) == ncclSuccess;
    }
    ok &= ncclGroupEnd() == ncclSuccess;
    if (!ok) {
      h->err = "RCCL send/recv group failed";
      return SWIM_EDEVICE;
    }
  }
  return SWIM_OK;
}

// one all-to-all of per-peer byte blocks (fixed-capacity regions of `cap` bytes in send / recv, rank order).
// The byte counts are device-resident (written by the pack kernels); the transport needs them on the host.
int exchange(swim_handle* h, uint8_t* send, uint8_t* recv, uint64_t cap, unsigned long long* scnt,
             unsigned long long* rcnt, bool inline_packed) {
  const uint32_t W = h->d.W;
  hipStream_t st = h->stream;
  unsigned long long* hc = h->hcnt;
  auto t0 = std::chrono::steady_clock::now();
  if (h->spec.transport == SWIM_TRANSPORT_RCCL) {
    // one fixed-size all-to-all (count word + the first XINL - 8 bytes of each region), one host read of the
    // count words through mapped memory, and a send/recv group only for regions that did not fit
    if (!inline_packed) launch_inline_out(h->d, send, cap, scnt, st);  // exchange A: k_pack_all wrote them
    int rc;
    if ((rc = exchange_inline(h, recv, cap, scnt, rcnt, false)) != SWIM_OK) return rc;
    HIPCK(hipEventRecord(h->ev_member, st));
    HIPCK(spin_wait(h->ev_member));
    if ((rc = exchange_rest(h, send, recv, cap)) != SWIM_OK) return rc;
  } else {
    HIPCK(hipMemcpyAsync(hc, scnt, 8ull * W, hipMemcpyDeviceToHost, st));
    HIPCK(hipStreamSynchronize(st));
    uint64_t off = 0;
    for (uint32_t q = 0; q < W; ++q) {
      const uint64_t sb = hc[q] & XCNT_MASK;
      if (sb > cap) {
        h->err = "exchange block larger than its region";
        return SWIM_ECAPACITY;
      }
      if (sb) HIPCK(hipMemcpyAsync(h->hsend.data() + off, send + (size_t)q * cap, sb, hipMemcpyDeviceToHost, st));
      off += sb;
    }
    HIPCK(hipStreamSynchronize(st));
    uint64_t sb[64], rb[64];
    for (uint32_t q = 0; q < W; ++q) sb[q] = hc[q], rb[q] = 0;
    if (h->spec.exchange(h->spec.ctx, h->hsend.data(), sb, h->hrecv.data(), h->hrecv.size(), rb) != 0) {
      h->err = "host exchange callback failed";
      return SWIM_EDEVICE;
    }
    off = 0;
    h->xflag = false;
    for (uint32_t p = 0; p < W; ++p) {
      const uint64_t n = rb[p] & XCNT_MASK;
      if (n > cap) {
        h->err = "received exchange block larger than its region";
        return SWIM_ECAPACITY;
      }
      if (n) HIPCK(hipMemcpyAsync(recv + (size_t)p * cap, h->hrecv.data() + off, n, hipMemcpyHostToDevice, st));
      off += n;
      hc[W + p] = rb[p];
      h->xflag |= ((rb[p] | sb[p]) & XFLAG_GOSSIP) != 0;
    }
    HIPCK(hipMemcpyAsync(rcnt, hc + W, 8ull * W, hipMemcpyHostToDevice, st));
    HIPCK(hipStreamSynchronize(st));
  }
  h->xchg_ms += std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
  return SWIM_OK;
}

// slot sharding: sum the shards' gossip-count deltas of this tick and apply them (k_held_add). RCCL: one in-place
// all-reduce on the stream. HOST: every shard sends its delta vector to every peer and sums what it receives.
int held_allreduce(swim_handle* h) {
  Dev& d = h->d;
  hipStream_t st = h->stream;
  auto t0 = std::chrono::steady_clock::now();
  if (h->lone) {
    launch_held_add(d, d.held_delta, st);
  } else if (h->spec.transport == SWIM_TRANSPORT_RCCL) {
    if (ncclAllReduce(d.held_delta, d.held_delta, d.N, ncclInt32, ncclSum, h->comm, st) != ncclSuccess) {
      h->err = "ncclAllReduce (gossip counts) failed";
      return SWIM_EDEVICE;
    }
    launch_held_add(d, d.held_delta, st);
  } else {
    const uint64_t bytes = 4ull * d.N;
    HIPCK(hipMemcpyAsync(h->hsend.data(), d.held_delta, bytes, hipMemcpyDeviceToHost, st));
    HIPCK(hipStreamSynchronize(st));
    for (uint32_t q = 1; q < d.XW; ++q) std::memcpy(h->hsend.data() + q * bytes, h->hsend.data(), bytes);
    uint64_t sb[64], rb[64];
    for (uint32_t q = 0; q < d.XW; ++q) sb[q] = q == d.xrank ? 0 : bytes, rb[q] = 0;
    if (h->spec.exchange(h->spec.ctx, h->hsend.data(), sb, h->hrecv.data(), h->hrecv.size(), rb) != 0) {
      h->err = "host exchange callback failed";
      return SWIM_EDEVICE;
    }
    std::vector<int32_t> sum((size_t)d.N);
    std::memcpy(sum.data(), h->hsend.data(), bytes);
    uint64_t off = 0;
    for (uint32_t p = 0; p < d.XW; ++p) {
      const uint64_t n = rb[p] & XCNT_MASK;
      if (n != (p == d.xrank ? 0 : bytes)) {
        h->err = "gossip-count exchange: unexpected block size";
        return SWIM_EDEVICE;
      }
      const int32_t* v = (const int32_t*)(h->hrecv.data() + off);
      for (uint32_t m = 0; m < n / 4; ++m) sum[m] += v[m];
      off += n;
    }
    HIPCK(hipMemcpyAsync(d.held_delta, sum.data(), bytes, hipMemcpyHostToDevice, st));
    launch_held_add(d, d.held_delta, st);
    HIPCK(hipStreamSynchronize(st));
  }
  h->xchg_ms += std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
  return SWIM_OK;
}

int create(const swim_config* cfg, const swim_shard_spec* spec, swim_handle** out) {
  if (!cfg || !out) return SWIM_EINVAL;
  *out = nullptr;
  const swim_config& c = *cfg;
  if (c.n_members < 2 || c.n_members > (1u << 20) || c.ping_timeout_ms >= c.ping_interval_ms || c.gossip_fanout == 0 || c.gossip_fanout > 8 ||
      c.ping_req_members > 8 || c.n_seeds > 16 || c.mode > SWIM_MODE_RUMOR ||
      (c.mode == SWIM_MODE_RUMOR && c.init_mode != SWIM_INIT_PRECONVERGED) || c.n_dormant > c.n_members ||
      (c.n_dormant && c.init_mode != SWIM_INIT_COLD_JOIN))
    return SWIM_EINVAL;
  if (c.latency_ticks != 1) return SWIM_EUNSUPPORTED;  // gossip data plane assumes one-tick hops
  if (spec) {
    if (spec->world < 1 || spec->world > 64 || spec->rank >= spec->world || spec->world > c.n_members / 2) return SWIM_EINVAL;
    if (spec->world > 1 && spec->transport != SWIM_TRANSPORT_RCCL &&
        !(spec->transport == SWIM_TRANSPORT_HOST && spec->exchange))
      return SWIM_EINVAL;
  }
  int ndev = 0;
  if (hipGetDeviceCount(&ndev) != hipSuccess || ndev <= (int)c.device) return SWIM_EDEVICE;
  auto* h = new swim_handle();
  h->cfg = c;
  if (spec) h->spec = *spec;
  if (h->spec.world == 0) h->spec.world = 1;
  if (hipSetDevice((int)c.device) != hipSuccess || hipStreamCreateWithFlags(&h->stream, hipStreamNonBlocking) != hipSuccess) {
    delete h;
    return SWIM_EDEVICE;
  }
  if (h->spec.world > 1 && h->spec.transport == SWIM_TRANSPORT_RCCL) {
    ncclUniqueId id;
    static_assert(sizeof(id) == 128, "ncclUniqueId size");
    std::memcpy(&id, h->spec.rccl_id, sizeof(id));
    if (ncclCommInitRank(&h->comm, (int)h->spec.world, id, (int)h->spec.rank) != ncclSuccess) {
      fprintf(stderr, "swim_create_sharded: ncclCommInitRank failed (rank %u of %u)\n", h->spec.rank, h->spec.world);
      h->comm = nullptr;
      swim_destroy(h);
      return SWIM_EDEVICE;
    }
  }
  int rc = build(h);
  if (rc != SWIM_OK) {
    fprintf(stderr, "swim_create: %s\n", h->err.c_str());
    swim_destroy(h);
    return rc;
  }
  *out = h;
  return SWIM_OK;
}

bool owns(const swim_handle* h, uint32_t m) { return m >= h->d.lo && m < h->d.hi; }

}  // namespace

// ---------------------------------------------------------------------------------------------------------------
// One handle over several GPUs (swim_config.n_gpus = W > 1; SURVEY.md §8b: "RCCL communicators created in
// swim_create", ClusterConfig unchanged for the caller). The handle owns W row-sharded shard handles
// (swimhip_shard.h), one per device, and forwards every call: stepping runs the shards on W host threads in
// lockstep; fault injection goes to every shard; readback goes to the owning shard (rows, lists, gossips) or is
// summed / merged over them (hashes, counters, events), exactly as a multi-process deployment would combine them.
// Transport: RCCL between W distinct devices (one communicator per shard, initialised together); on a node with
// fewer devices (the single-GPU test box) the shards share the devices and exchange through host memory inside this
// process (SWIM_GROUP_HOST=1 forces that).
struct Group {
  std::vector<swim_handle*> shards;
  std::vector<uint32_t> lo, hi;
  uint32_t transport = SWIM_TRANSPORT_HOST;
  // in-process host exchange: each rank deposits its blocks, waits for all, copies its own, waits again
  std::mutex mu;
  std::condition_variable cv;
  uint32_t arrived = 0;
  uint64_t gen = 0;
  bool abort = false;
  struct Block {
    const uint8_t* data = nullptr;
    std::vector<uint64_t> words;
  };
  std::vector<Block> blocks;
  struct End {
    Group* g;
    uint32_t rank;
  };
  std::vector<End> ends;
  std::vector<swim_event> events;
  bool slots = false;             // slot-sharded (RUMOR mode): every shard runs every member, gossips are split
  std::vector<uint32_t> evcount;  // slot-sharded: events per observer drained so far (the merged seq)
};

namespace {

bool group_barrier(Group* g) {
  std::unique_lock<std::mutex> lk(g->mu);
  if (g->abort) return false;
  const uint64_t my = g->gen;
  if (++g->arrived == g->shards.size()) {
    g->arrived = 0;
    g->gen++;
    g->cv.notify_all();
    return true;
  }
  const bool ok = g->cv.wait_for(lk, std::chrono::seconds(600), [&] { return g->gen != my || g->abort; });
  return ok && !g->abort;
}

void group_abort(Group* g) {
  std::lock_guard<std::mutex> lk(g->mu);
  g->abort = true;
  g->cv.notify_all();
}

// swim_exchange_fn of the in-process transport (the contract of swimhip_shard.h)
int group_exchange(void* ctx, const void* send, const uint64_t* sb, void* recv, uint64_t cap, uint64_t* rb) {
  const Group::End* e = (const Group::End*)ctx;
  Group* g = e->g;
  const uint32_t W = (uint32_t)g->shards.size(), r = e->rank;
  g->blocks[r].data = (const uint8_t*)send;
  g->blocks[r].words.assign(sb, sb + W);
  if (!group_barrier(g)) return -1;
  uint64_t out = 0;
  for (uint32_t p = 0; p < W; ++p) {
    const Group::Block& B = g->blocks[p];
    uint64_t off = 0;
    for (uint32_t q = 0; q < r; ++q) off += B.words[q] & SWIM_XCOUNT_MASK;
    const uint64_t n = B.words[r] & SWIM_XCOUNT_MASK;
    if (out + n > cap) {
      group_abort(g);
      return -1;
    }
    if (n) std::memcpy((uint8_t*)recv + out, B.data + off, n);
    out += n;
    rb[p] = B.words[r];
  }
  return group_barrier(g) ? 0 : -1;  // every peer has copied before the send buffers are reused
}

int fail(swim_handle* h, int rc, const std::string& what) {
  h->err = what;
  return rc;
}

int create_group(const swim_config* cfg, swim_handle** out) {
  const uint32_t W = cfg->n_gpus;
  if (W > 64 || W > cfg->n_members / 2) return SWIM_EINVAL;
  int ndev = 0;
  if (hipGetDeviceCount(&ndev) != hipSuccess || ndev <= (int)cfg->device) return SWIM_EDEVICE;
  auto* h = new swim_handle();
  h->cfg = *cfg;
  Group* g = h->grp = new Group();
  const bool rccl = (uint64_t)cfg->device + W <= (uint64_t)ndev && !getenv("SWIM_GROUP_HOST");
  g->transport = rccl ? SWIM_TRANSPORT_RCCL : SWIM_TRANSPORT_HOST;
  g->shards.assign(W, nullptr);
  g->blocks.resize(W);
  for (uint32_t r = 0; r < W; ++r) g->ends.push_back(Group::End{g, r});
  std::vector<int> rc(W, SWIM_OK);
  auto make = [&](uint32_t r, const uint8_t* id) {
    swim_config c = *cfg;
    c.n_gpus = 1;
    c.device = rccl ? cfg->device + r : cfg->device + r % (uint32_t)(ndev - (int)cfg->device);
    swim_shard_spec sp{};
    sp.rank = r;
    sp.world = W;
    sp.transport = g->transport;
    if (rccl) {
      std::memcpy(sp.rccl_id, id, 128);
    } else {
      sp.exchange = group_exchange;
      sp.ctx = &g->ends[r];
    }
    rc[r] = create(&c, &sp, &g->shards[r]);
  };
  if (rccl) {  // ncclCommInitRank is collective: every rank's call runs on its own thread
    ncclUniqueId id;
    if (ncclGetUniqueId(&id) != ncclSuccess) {
      swim_destroy(h);
      return SWIM_EDEVICE;
    }
    std::vector<std::thread> th;
    for (uint32_t r = 0; r < W; ++r) th.emplace_back(make, r, (const uint8_t*)&id);
    for (auto& t : th) t.join();
  } else {
    for (uint32_t r = 0; r < W; ++r) make(r, nullptr);
  }
  for (uint32_t r = 0; r < W; ++r)
    if (rc[r] != SWIM_OK) {
      swim_destroy(h);
      return rc[r];
    }
  for (swim_handle* s : g->shards) {
    g->lo.push_back(s->d.lo);
    g->hi.push_back(s->d.hi);
  }
  g->slots = g->shards[0]->d.XW > 1;
  g->evcount.assign(g->slots ? cfg->n_members : 0, 0);
  h->d = g->shards[0]->d;  // constants only (N, ping_t, ...): the group handle itself launches nothing
  *out = h;
  return SWIM_OK;
}

// run f on every shard (on its device), in rank order; the first error is the group's
template <class F>
int group_all(swim_handle* h, F f) {
  Group* g = h->grp;
  for (size_t r = 0; r < g->shards.size(); ++r) {
    hipSetDevice((int)g->shards[r]->cfg.device);
    const int rc = f(g->shards[r]);
    if (rc != SWIM_OK) return fail(h, rc, "shard " + std::to_string(r) + ": " + g->shards[r]->err);
  }
  return SWIM_OK;
}

// run f on the shard that owns observer m
template <class F>
int group_owner(swim_handle* h, uint32_t m, F f) {
  Group* g = h->grp;
  for (size_t r = 0; r < g->shards.size(); ++r)
    if (m >= g->lo[r] && m < g->hi[r]) {
      hipSetDevice((int)g->shards[r]->cfg.device);
      const int rc = f(g->shards[r]);
      if (rc != SWIM_OK) return fail(h, rc, "shard " + std::to_string(r) + ": " + g->shards[r]->err);
      return rc;
    }
  return SWIM_EINVAL;
}

}  // namespace

#define GROUP_ALL(call)                                            \
  if (h && h->grp) return group_all(h, [&](swim_handle* s) { return call; })
#define GROUP_OWNER(m, call)                                       \
  if (h && h->grp) return group_owner(h, (m), [&](swim_handle* s) { return call; })

extern "C" {

uint32_t swim_abi_version(void) { return SWIM_ABI_VERSION; }

void swim_default_config(swim_config* c) {
  std::memset(c, 0, sizeof(*c));
  c->tick_ms = 100;
  c->latency_ticks = 1;
  c->init_mode = SWIM_INIT_PRECONVERGED;
  c->seed = 0x5EED5EEDull;
  c->sync_interval_ms = 30000;
  c->sync_timeout_ms = 3000;
  c->suspicion_mult = 5;
  c->ping_interval_ms = 1000;
  c->ping_timeout_ms = 500;
  c->ping_req_members = 3;
  c->gossip_interval_ms = 200;
  c->gossip_fanout = 3;
  c->gossip_repeat_mult = 3;
  c->metadata_timeout_ms = 3000;
  c->n_gpus = 1;
}

int swim_is_overrides(uint32_t s1, uint32_t i1, uint32_t s0, uint32_t i0) { return overrides(s1, i1, s0, i0) ? 1 : 0; }
uint32_t swim_ceil_log2(uint32_t n) { return bitlen(n); }

int swim_create(const swim_config* cfg, swim_handle** out) {
  // one handle for all N observers: on one GPU, or row-sharded over n_gpus devices inside this process (Group)
  if (cfg && out && cfg->n_gpus > 1) {
    *out = nullptr;
    return create_group(cfg, out);
  }
  return create(cfg, nullptr, out);
}

int swim_create_sharded(const swim_config* cfg, const swim_shard_spec* spec, swim_handle** out) {
  if (!spec) return SWIM_EINVAL;
  return create(cfg, spec, out);
}

int swim_rccl_unique_id(uint8_t* out128) {
  if (!out128) return SWIM_EINVAL;
  ncclUniqueId id;
  if (ncclGetUniqueId(&id) != ncclSuccess) return SWIM_EDEVICE;
  std::memcpy(out128, &id, 128);
  return SWIM_OK;
}

int swim_shard_range(swim_handle* h, uint32_t* lo, uint32_t* hi) {
  if (!h || !lo || !hi) return SWIM_EINVAL;
  if (h->grp) {  // the group reports on every observer
    *lo = 0;
    *hi = h->d.N;
    return SWIM_OK;
  }
  *lo = h->d.lo;
  *hi = h->d.hi;
  return SWIM_OK;
}

int swim_destroy(swim_handle* h) {
  if (!h) return SWIM_EINVAL;
  if (h->grp) {
    for (swim_handle* s : h->grp->shards)
      if (s) swim_destroy(s);
    delete h->grp;
    delete h;
    return SWIM_OK;
  }
  hipSetDevice((int)h->cfg.device);
  if (h->stream) hipStreamSynchronize(h->stream);
  for (void* p : h->allocs) hipFree(p);
  for (auto& te : h->prof)
    for (auto& e : te.ev) hipEventDestroy((hipEvent_t)e);
  if (h->comm) ncclCommDestroy(h->comm);
  if (h->hcnt) hipHostFree(h->hcnt);
  if (h->hflag) hipHostFree((void*)h->hflag);
  if (h->xi_host_h) hipHostFree(h->xi_host_h);
  if (h->ev_member) hipEventDestroy(h->ev_member);
  if (h->stream) hipStreamDestroy(h->stream);
  delete h;
  return SWIM_OK;
}

// W == 1 with SWIM_FLAG_PROFILE: every DIFF_SAMPLE-th tick's k_sync_diff is bracketed by events (the roofline's
// sample); SWIM_DIFF_SAMPLE overrides it (measurements of the sampling's own cost)
static uint64_t diff_sample() {
  static const uint64_t v = [] {
    const char* e = getenv("SWIM_DIFF_SAMPLE");
    const unsigned long x = e ? strtoul(e, nullptr, 0) : 0ul;
    return x >= 1 && x <= 1000 ? (uint64_t)x : (uint64_t)10;
  }();
  return v;
}

int swim_step(swim_handle* h, uint32_t n) {
  if (!h) return SWIM_EINVAL;
  if (h->grp) {  // the shards in lockstep, one host thread each (their exchanges meet inside swim_step)
    Group* g = h->grp;
    std::vector<int> rc(g->shards.size(), SWIM_OK);
    std::vector<std::thread> th;
    for (size_t r = 0; r < g->shards.size(); ++r)
      th.emplace_back([&, r] {
        rc[r] = swim_step(g->shards[r], n);
        if (rc[r] != SWIM_OK) group_abort(g);  // peers waiting in an exchange give up
      });
    for (auto& t : th) t.join();
    h->tick = g->shards[0]->tick;
    for (size_t r = 0; r < rc.size(); ++r)
      if (rc[r] != SWIM_OK && g->shards[r]->err.size())
        return fail(h, rc[r], "shard " + std::to_string(r) + ": " + g->shards[r]->err);
    for (size_t r = 0; r < rc.size(); ++r)
      if (rc[r] != SWIM_OK) return fail(h, rc[r], "shard " + std::to_string(r) + " failed in a peer's exchange");
    return SWIM_OK;
  }
  hipSetDevice((int)h->cfg.device);
  if (h->tick + n >= (1ull << 28)) return SWIM_ECAPACITY;  // deadlines are stored in 29 bits
  const bool profile = (h->cfg.flags & (SWIM_FLAG_PROFILE | SWIM_FLAG_PROFILE_ALL)) != 0;
  if (profile)
    while (h->prof.size() < n) {
      TickEvents te;
      te.all = (h->cfg.flags & SWIM_FLAG_PROFILE_ALL) ? 1 : 0;
      for (auto& e : te.ev) HIPCK(hipEventCreate((hipEvent_t*)&e));
      h->prof.push_back(te);
    }
  uint64_t first = h->tick;
  const Dev& d = h->d;
  // W == 1 with SWIM_FLAG_PROFILE: only every diff_sample()-th tick's k_sync_diff is bracketed by events (an event
  // pair costs GPU time of its own); the timed launches count their own messages (diff_msgs)
  const uint64_t ds = diff_sample();
  auto timed = [&](uint64_t kk) {
    return profile && ((h->cfg.flags & SWIM_FLAG_PROFILE_ALL) || d.W > 1 || kk % ds == 0);
  };
  bool need_diff = true;  // W == 1: SYNC diff(k) not queued yet (it is queued with the previous tick when it can be)
  for (uint32_t i = 0; i < n;) {
    const TickEvents* te = timed(h->tick) ? &h->prof[i] : nullptr;
    const uint32_t k = (uint32_t)h->tick;
    if (h->tick >= h->next_scrub) {  // stale holder entries of recycled slots, before they can alias (engine.h)
      launch_s_scrub(d, k, h->stream);
      h->next_scrub = h->tick + SCRUB;
    }
    // a speculative batch ends at the next scrub tick
    const uint32_t nb = (uint32_t)std::min<uint64_t>(n, i + (h->next_scrub - h->tick));
    // P0 gossip creations before the member kernel: RUMOR-mode churn rumors, then the user gossips queued by the host
    if (d.churn && k % d.ping_t == 0) launch_churn(d, k, h->stream);
    if (i == 0 && !h->ugq.empty()) {
      const size_t pairs = h->ugq.size() / 2;
      if (pairs > h->ug_cap) {
        int rc;
        h->ug_cap = std::max<size_t>(pairs, 1024);
        if ((rc = dalloc(h, &h->ug_dev, 2 * h->ug_cap)) != SWIM_OK) return rc;
      }
      HIPCK(hipMemcpyAsync(h->ug_dev, h->ugq.data(), h->ugq.size() * 8, hipMemcpyHostToDevice, h->stream));
      launch_user_gossips(d, k, h->ug_dev, (uint32_t)pairs, h->stream);
      HIPCK(hipStreamSynchronize(h->stream));  // the host queue is reused after this
      h->ugq.clear();
    }
    if (d.W == 1 && h->gossip_idle && i + 1 < nb && d.XW == 1 && !d.churn && !h->no_pipe && !h->no_skip &&
        !h->no_spec && !(h->cfg.flags & SWIM_FLAG_PROFILE_ALL)) {  // (PROFILE_ALL times every tick's gossip plane)
      // Speculative batch: while no gossip slot is in use the host need not look at the flag after every member
      // kernel. The rest of the call is queued as diff / member pairs with no host wait; the member kernel after which
      // a slot is in use raises d.halt, every later launch of the batch returns at once, and the host resumes after
      // that tick with the gossip plane.
      for (uint32_t j = i; j < nb; ++j) {
        const uint32_t kj = k + (j - i);
        if (need_diff) launch_diff(d, kj, h->stream, timed(kj) ? &h->prof[j] : nullptr, true);
        launch_member(d, kj, h->stream, timed(kj) ? &h->prof[j] : nullptr, true);
        need_diff = j + 1 == nb;
        if (!need_diff) launch_diff(d, kj + 1, h->stream, timed(kj + 1ull) ? &h->prof[j + 1] : nullptr, true);
      }
      HIPCK(hipMemcpyAsync((void*)(h->hflag + 1), d.halt, 4, hipMemcpyDeviceToHost, h->stream));
      HIPCK(hipStreamSynchronize(h->stream));
      const uint32_t hk = h->hflag[1];
      if (hk == 0) {  // the whole batch ran
        h->tick += nb - i;
        i = nb;
        h->gossip_ran = false;
        continue;
      }
      const uint32_t kh = hk - 1u;  // member(kh) ran; the launches after it returned at once
      if (kh < k || kh >= k + (nb - i)) return fail(h, SWIM_EDEVICE, "speculative batch: bad halt tick");
      HIPCK(hipMemsetAsync(d.halt, 0, 4, h->stream));
      const uint32_t ih = i + (kh - k);
      // a speculative member launch publishes no flag (tick_flag): the slots in use after member(kh) are read here, so
      // the first gossip plane after an idle stretch gets the same capacity check as every other one (grow_caps); the
      // device copy of the flag word follows, so tick_flag keeps writing it only on a change
      {
        int32_t top = 0;
        HIPCK(hipMemcpyAsync(&top, d.free_top, 4, hipMemcpyDeviceToHost, h->stream));
        HIPCK(hipStreamSynchronize(h->stream));
        const uint32_t used = (uint32_t)((int32_t)d.SPR - top);
        h->hflag[0] = used;
        HIPCK(hipMemcpyAsync(d.hsh, &used, 4, hipMemcpyHostToDevice, h->stream));
        int gr;
        if ((gr = grow_caps(h)) != SWIM_OK) return gr;
      }
      launch_gossip(d, kh, h->stream, timed(kh) ? &h->prof[ih] : nullptr);
      h->gossip_idle = false;
      h->gossip_ran = true;
      need_diff = true;  // diff(kh + 1) returned at once
      h->tick = kh + 1ull;
      i = ih + 1;
      continue;
    }
    if (d.W == 1) {
      // SYNC diff(k) was queued in the previous iteration, except for the first tick of this call
      if (need_diff) launch_diff(d, k, h->stream, te);
      launch_member(d, k, h->stream, te, false, h->gossip_ran && !d.fastp4);
      const bool nosync = (d.exp & 256) != 0;  // timing experiment: no per-tick event (gossip plane never launched)
      if (!nosync) HIPCK(hipEventRecord(h->ev_member, h->stream));
      const bool pipe = i + 1 < n && !h->no_pipe;
      if (pipe) launch_diff(d, k + 1, h->stream, timed(k + 1ull) ? &h->prof[i + 1] : nullptr);  // overlaps the wait
      need_diff = !pipe;
      if (!nosync) HIPCK(hipEventSynchronize(h->ev_member));  // (a spin wait measured the same here: diff(k+1) hides the wake-up)
      h->gossip_idle = !nosync && h->hflag[0] == 0;
      if (!nosync && !h->gossip_idle) {  // slots, rings and receipt lists sized up before they can overflow
        int gr;
        if ((gr = grow_caps(h)) != SWIM_OK) return gr;
      }
      h->gossip_ran = !nosync && (h->hflag[0] != 0 || h->no_skip);
      if (nosync) {
      } else if (h->hflag[0] != 0 || h->no_skip) {
        launch_gossip(d, k, h->stream, te);
        if (h->stats) {
          uint32_t v[8];
          HIPCK(hipStreamSynchronize(h->stream));
          const uint32_t* src[8] = {d.rc_n, d.ntl, d.nagroup, d.rp_n, d.slow_n, d.ncfl, d.nrx, d.nrwl};
          for (int q = 0; q < 8; ++q) HIPCK(hipMemcpy(&v[q], src[q], 4, hipMemcpyDeviceToHost));
          std::vector<uint32_t> rc(d.N), nf(d.N);
          HIPCK(hipMemcpy(rc.data(), d.rc_cnt, 4ull * d.N, hipMemcpyDeviceToHost));
          HIPCK(hipMemcpy2D(nf.data(), 4, &d.ms[0].nfetch, sizeof(MS), 4, d.N, hipMemcpyDeviceToHost));
          std::sort(rc.begin(), rc.end());
          std::sort(nf.begin(), nf.end());
          // first receipts per target with senders this tick (rtail - rt0), and senders per target
          std::vector<uint32_t> tl(v[1]), r0(d.N), r1(d.N), tc(d.N), fr, sn;
          HIPCK(hipMemcpy(tl.data(), d.tlist, 4ull * v[1], hipMemcpyDeviceToHost));
          HIPCK(hipMemcpy(r0.data(), d.rt0, 4ull * d.N, hipMemcpyDeviceToHost));
          HIPCK(hipMemcpy(r1.data(), d.rtail, 4ull * d.N, hipMemcpyDeviceToHost));
          HIPCK(hipMemcpy(tc.data(), d.tin_off, 4ull * d.N, hipMemcpyDeviceToHost));  // (tin_cnt is reset by then)
          uint64_t tot = 0;
          for (uint32_t t : tl) {
            fr.push_back(r1[t] - r0[t]);
            if (t + 1 < d.N) sn.push_back(tc[t + 1] - tc[t]);
            tot += r1[t] - r0[t];
          }
          std::sort(fr.begin(), fr.end());
          std::sort(sn.begin(), sn.end());
          const size_t nt = fr.size();
          fprintf(stderr, "stats tick %u: routed %u targets %u groups %u replay %u slow %u contacts %u rx %u rounds %u; "
                  "receipts per member median %u p99 %u max %u; pending fetches median %u p99 %u max %u; "
                  "first receipts %llu, per target median %u p90 %u p99 %u max %u; senders per target median %u max %u\n",
                  k, v[0], v[1], v[2], v[3], v[4], v[5], v[6], v[7], rc[d.N / 2], rc[d.N * 99 / 100], rc[d.N - 1],
                  nf[d.N / 2], nf[d.N * 99 / 100], nf[d.N - 1], (unsigned long long)tot, nt ? fr[nt / 2] : 0,
                  nt ? fr[nt * 9 / 10] : 0, nt ? fr[nt * 99 / 100] : 0, nt ? fr[nt - 1] : 0, sn.empty() ? 0 : sn[sn.size() / 2],
                  sn.empty() ? 0 : sn.back());
        }
      } else if (te && te->all) {
        HIPCK(hipEventRecord((hipEvent_t)te->ev[4], h->stream));
        HIPCK(hipEventRecord((hipEvent_t)te->ev[5], h->stream));
      }
      if (d.XW > 1) {  // slot sharding: the members' gossip counts, every tick (collective)
        int xr;
        if ((xr = held_allreduce(h)) != SWIM_OK) return xr;
      }
    } else if (h->spec.transport == SWIM_TRANSPORT_RCCL && !h->xflag && i + 1 < nb && !d.churn && !h->no_spec &&
               !(h->cfg.flags & SWIM_FLAG_PROFILE_ALL)) {
      // Speculative sharded batch: while no shard has a gossip slot in use and every exchange-A region fits its inline
      // block, a tick needs nothing from the host. The rest of the call is queued as A / inline all-to-all / B with
      // no host wait; the gate after the all-to-all of the first tick that needs the host (the same tick on every
      // shard: the flags ride on the exchanged count words) raises d.halt, every later launch returns at once (the
      // all-to-alls still run, carrying nothing anyone reads), and the host finishes that tick on the normal path.
      int xr;
      for (uint32_t j = i; j < nb; ++j) {
        const uint32_t kj = k + (j - i);
        const TickEvents* tj = timed(kj) ? &h->prof[j] : nullptr;
        launch_tick_a(d, kj, h->stream, tj, true);
        if ((xr = exchange_inline(h, d.xa_recv, d.XA_PEER, d.xa_scnt, d.xa_rcnt, true)) != SWIM_OK) return xr;
        launch_tick_b(d, kj, h->stream, tj, false, true);
      }
      HIPCK(hipMemcpyAsync((void*)(h->hflag + 1), d.halt, 4, hipMemcpyDeviceToHost, h->stream));
      HIPCK(hipStreamSynchronize(h->stream));
      const uint32_t hk = h->hflag[1];
      if (hk == 0) {
        h->tick += nb - i;
        i = nb;
        continue;
      }
      const uint32_t kh = hk - 1u;  // tick kh ran up to its inline exchange; the launches after that returned at once
      if (kh < k || kh >= k + (nb - i)) return fail(h, SWIM_EDEVICE, "speculative sharded batch: bad halt tick");
      HIPCK(hipMemsetAsync(d.halt, 0, 4, h->stream));
      const uint32_t ih = i + (kh - k);
      const TickEvents* th = timed(kh) ? &h->prof[ih] : nullptr;
      if ((xr = exchange_rest(h, d.xa_send, d.xa_recv, d.XA_PEER)) != SWIM_OK) return xr;
      const bool gossip = h->xflag;
      launch_tick_b(d, kh, h->stream, th, gossip);
      if (gossip && (xr = exchange(h, d.xb_send, d.xb_recv, d.XB_PEER, d.xb_scnt, d.xb_rcnt, false)) != SWIM_OK) return xr;
      launch_tick_c(d, kh, h->stream, gossip);
      if (gossip && (xr = grow_caps_shard(h)) != SWIM_OK) return xr;
      h->tick = kh + 1ull;
      i = ih + 1;
      continue;
    } else {
      int xr;
      launch_tick_a(d, k, h->stream, te);
      if ((xr = exchange(h, d.xa_send, d.xa_recv, d.XA_PEER, d.xa_scnt, d.xa_rcnt, true)) != SWIM_OK) return xr;
      const bool gossip = h->xflag;
      launch_tick_b(d, k, h->stream, te, gossip);
      if (gossip && (xr = exchange(h, d.xb_send, d.xb_recv, d.XB_PEER, d.xb_scnt, d.xb_rcnt, false)) != SWIM_OK) return xr;
      launch_tick_c(d, k, h->stream, gossip);
      if (gossip && (xr = grow_caps_shard(h)) != SWIM_OK) return xr;
    }
    h->tick++;
    ++i;
  }
  int rc = check_err(h);
  if (rc == SWIM_OK && (d.exp & (16 | 128))) {  // timing experiments: member-kernel shader cycles per phase since the last step (16: sum over members, 128: max)
    unsigned long long c[5];
    HIPCK(hipMemcpy(c, d.ctr + 8, sizeof(c), hipMemcpyDeviceToHost));
    HIPCK(hipMemset(d.ctr + 8, 0, sizeof(c)));
    fprintf(stderr, "exp: member cycles P0+P1 %llu P2+P3 %llu P4 %llu P5 %llu P6 %llu\n", c[0], c[1], c[2], c[3], c[4]);
    if (d.exp & 128) {
      unsigned long long w[2];
      HIPCK(hipMemcpy(w, d.ctr + 14, sizeof(w), hipMemcpyDeviceToHost));
      HIPCK(hipMemset(d.ctr + 14, 0, sizeof(w)));
      fprintf(stderr, "exp: SYNC full walks %llu, largest candidate count %llu\n", w[0], w[1]);
    }
  }
  if (rc == SWIM_OK && (d.exp & 512)) {  // timing experiment: per-wave wall clock of the latest member kernel
    const size_t nw = (size_t)(d.NL + 255) / 256 * 4;
    std::vector<unsigned long long> w16(nw * 16), w(nw * 4);
    HIPCK(hipMemcpy(w16.data(), d.wt, w16.size() * 8, hipMemcpyDeviceToHost));
    for (size_t i = 0; i < nw; ++i)
      for (int j = 0; j < 4; ++j) w[4 * i + j] = w16[16 * i + j];
    const unsigned long long M = (1ull << 48) - 1;
    unsigned long long t0 = ~0ull, tend = 0;
    for (size_t i = 0; i < nw; ++i) t0 = std::min(t0, w[4 * i]), tend = std::max(tend, w[4 * i + 3]);
    std::vector<size_t> ord(nw);
    for (size_t i = 0; i < nw; ++i) ord[i] = i;
    // the waves whose bodies end last (a block's waves also wait for each other at the deferred copy-on-write)
    std::sort(ord.begin(), ord.end(), [&](size_t a, size_t b) { return w[4 * a + 2] > w[4 * b + 2]; });
    double sst = 0, str = 0, sbd = 0, scw = 0;
    for (size_t i = 0; i < nw; ++i) {
      sst += (double)(w[4 * i] - t0), str += (double)((w[4 * i + 1] & M) - w[4 * i]);
      sbd += (double)(w[4 * i + 2] - (w[4 * i + 1] & M)), scw += (double)(w[4 * i + 3] - w[4 * i + 2]);
    }
    fprintf(stderr, "exp512: span %.2f us; mean per wave (us): start %.2f triage %.2f body %.2f cow %.2f\n",
            (tend - t0) / 100.0, sst / nw / 100.0, str / nw / 100.0, sbd / nw / 100.0, scw / nw / 100.0);
    for (size_t r = 0; r < 8 && r < nw; ++r) {
      const size_t i = ord[r];
      if (r == 0) {  // when the waves of each class finish their bodies (us from the kernel's first wave): quartiles
        for (int c = 0; c < 4; ++c) {
          std::vector<double> e;
          for (size_t j = 0; j < nw; ++j)
            if ((w[4 * j + 1] >> 56) == (1ull << c)) e.push_back((w[4 * j + 2] - t0) / 100.0);
          std::sort(e.begin(), e.end());
          if (!e.empty())
            fprintf(stderr, "exp512: class %d waves %zu body end min %.1f q1 %.1f med %.1f q3 %.1f max %.1f\n", c, e.size(),
                    e[0], e[e.size() / 4], e[e.size() / 2], e[3 * e.size() / 4], e.back());
        }
      }
      fprintf(stderr, "exp512: wave %zu start %.2f triage %.2f body %.2f cow %.2f classes %llx busy %llu\n", i,
              (w[4 * i] - t0) / 100.0, ((w[4 * i + 1] & M) - w[4 * i]) / 100.0, (w[4 * i + 2] - (w[4 * i + 1] & M)) / 100.0,
              (w[4 * i + 3] - w[4 * i + 2]) / 100.0, w[4 * i + 1] >> 56, (w[4 * i + 1] >> 48) & 255);
      if (w[4 * i + 1] >> 56) {  // its lead lane's laps in time order, "slot:us since the previous lap"
        // (slots 0-4: after P0+P1, P2+P3, P4, P5, P6; 5-11: finer laps inside them)
        unsigned long long prev = w[4 * i + 1] & M;
        std::vector<std::pair<unsigned long long, int>> laps;
        for (int j = 0; j < 12; ++j)
          if (w16[16 * i + 4 + j] >= prev && w16[16 * i + 4 + j] <= w[4 * i + 2]) laps.push_back({w16[16 * i + 4 + j], j});
        std::sort(laps.begin(), laps.end());
        fprintf(stderr, "exp512:   laps");
        for (const auto& l : laps)
          fprintf(stderr, " %d:%.2f@%.1f", l.second, (l.first - prev) / 100.0, (l.first - t0) / 100.0), prev = l.first;
        fprintf(stderr, "\n");
      }
    }
  }
  if (rc == SWIM_OK && (d.exp & 4)) {  // timing experiments: gossip-send work counters since the last step
    unsigned long long c[5], u[2];
    HIPCK(hipMemcpy(c, d.ctr + 8, sizeof(c), hipMemcpyDeviceToHost));
    HIPCK(hipMemset(d.ctr + 8, 0, sizeof(c)));
    HIPCK(hipMemcpy(u, d.ctr + C_XU, sizeof(u), hipMemcpyDeviceToHost));
    HIPCK(hipMemset(d.ctr + C_XU, 0, sizeof(u)));
    fprintf(stderr, "exp: items %llu contact-bits %llu replayed %llu candidates %llu blocked %llu target-group items %llu "
            "sender words %llu\n", c[0], c[1], c[2], c[3], c[4], u[0], u[1]);
  }
  if (rc == SWIM_OK && profile) {
    for (uint32_t i = 0; i < n; ++i) {
      float ms = 0;
      if (!timed(first + i)) continue;
      if (first + i > 0) {
        HIPCK(hipEventElapsedTime(&ms, (hipEvent_t)h->prof[i].ev[0], (hipEvent_t)h->prof[i].ev[1]));
        h->prof_ms[0] += ms;
        h->prof_diff_launches++;
      }
      if (!h->prof[i].all) continue;
      HIPCK(hipEventElapsedTime(&ms, (hipEvent_t)h->prof[i].ev[2], (hipEvent_t)h->prof[i].ev[3]));
      h->prof_ms[1] += ms;
      HIPCK(hipEventElapsedTime(&ms, (hipEvent_t)h->prof[i].ev[4], (hipEvent_t)h->prof[i].ev[5]));
      h->prof_ms[2] += ms;
    }
  }
  return rc;
}

int swim_run_periods(swim_handle* h, uint32_t n) {
  if (!h) return SWIM_EINVAL;
  return swim_step(h, n * h->d.ping_t);
}

int swim_sync(swim_handle* h) {
  GROUP_ALL(swim_sync(s));
  return h ? check_err(h) : SWIM_EINVAL;
}

int swim_kill(swim_handle* h, uint32_t m) {
  GROUP_ALL(swim_kill(s, m));
  if (!h || m >= h->d.N) return SWIM_EINVAL;
  uint32_t t = (uint32_t)h->tick;
  HIPCK(hipMemcpyAsync(h->d.dead_tick + m, &t, 4, hipMemcpyHostToDevice, h->stream));
  // (the crashed member's holder state stays as it is: it never sends again, sends to it fail, and its slots expire)
  return check_err(h);
}

int swim_join(swim_handle* h, uint32_t m, const uint32_t* seeds, uint32_t n) {
  GROUP_ALL(swim_join(s, m, seeds, n));
  if (!h || m >= h->d.N || n > 16 || (n && !seeds)) return SWIM_EINVAL;
  if (m < h->d.N - h->d.n_dormant) return SWIM_EINVAL;  // only a dormant member starts later
  if (h->joined.empty()) h->joined.assign(h->d.N, 0);
  if (h->joined[m]) return SWIM_EINVAL;
  h->joined[m] = 1;
  uint32_t sd[16], ns = 0;  // LinkedHashSet of valid ids minus self (MembershipProtocolImpl.java:160-166)
  for (uint32_t i = 0; i < n; ++i) {
    bool dup = seeds[i] >= h->d.N || seeds[i] == m;
    for (uint32_t j = 0; j < ns; ++j) dup |= sd[j] == seeds[i];
    if (!dup) sd[ns++] = seeds[i];
  }
  launch_join(h->d, m, (uint32_t)h->tick, sd, ns, h->stream);  // every shard: the arrays are replicated
  return check_err(h);
}

int swim_spread_gossip(swim_handle* h, uint32_t m, uint64_t payload) {
  GROUP_ALL(swim_spread_gossip(s, m, payload));
  if (!h || m >= h->d.N) return SWIM_EINVAL;
  if (!owns(h, m)) return SWIM_OK;  // the owning shard creates it; the others receive its slot in exchange A
  uint32_t dt = 0;
  HIPCK(hipStreamSynchronize(h->stream));
  HIPCK(hipMemcpy(&dt, h->d.dead_tick + m, 4, hipMemcpyDeviceToHost));
  if (dt != NEVER) return SWIM_EINVAL;
  h->ugq.push_back(m);
  h->ugq.push_back(payload);
  return SWIM_OK;
}

int swim_update_metadata(swim_handle* h, uint32_t m) {
  GROUP_ALL(swim_update_metadata(s, m));
  if (!h || m >= h->d.N) return SWIM_EINVAL;
  if (h->d.implicit) return SWIM_EUNSUPPORTED;  // implicit views: the tables are not stored
  uint32_t dt = 0, ver = 0;
  HIPCK(hipStreamSynchronize(h->stream));
  HIPCK(hipMemcpy(&dt, h->d.dead_tick + m, 4, hipMemcpyDeviceToHost));
  if (dt != NEVER) return SWIM_EINVAL;
  if (std::find(h->md_cols.begin(), h->md_cols.end(), m) == h->md_cols.end()) {
    if (h->md_cols.size() >= MDU) {
      h->err = "swim_update_metadata: more than " + std::to_string(MDU) + " members with updated metadata";
      return SWIM_ECAPACITY;
    }
    launch_md_column(h->d, m, (uint32_t)h->md_cols.size(), h->stream);
    h->md_cols.push_back(m);
    HIPCK(hipStreamSynchronize(h->stream));
  }
  // every shard keeps the versions of all members (responses are evaluated at the issuer's shard)
  HIPCK(hipMemcpy(&ver, h->d.md_version + m, 4, hipMemcpyDeviceToHost));
  ++ver;
  HIPCK(h2d(h->stream, h->d.md_version + m, &ver, 4));
  return swim_update_incarnation(h, m);
}

int swim_update_incarnation(swim_handle* h, uint32_t m) {
  GROUP_ALL(swim_update_incarnation(s, m));
  if (!h || m >= h->d.N) return SWIM_EINVAL;
  if (h->d.implicit) return SWIM_EUNSUPPORTED;  // implicit views: the tables are not stored
  if (!owns(h, m)) return SWIM_OK;  // the owning shard bumps it; the others learn it from its gossip
  uint32_t req = 0, dt = 0;
  HIPCK(hipStreamSynchronize(h->stream));
  HIPCK(hipMemcpy(&dt, h->d.dead_tick + m, 4, hipMemcpyDeviceToHost));
  if (dt != NEVER) return SWIM_EINVAL;
  HIPCK(hipMemcpy(&req, h->d.pending_inc + m, 4, hipMemcpyDeviceToHost));
  req += 4u;  // bits 2..: incarnation bumps requested (one per call), bit 1: leave
  HIPCK(h2d(h->stream, h->d.pending_inc + m, &req, 4));
  return SWIM_OK;
}

// MembershipProtocolImpl.leaveCluster (:197-206) via ClusterImpl.shutdown -> doShutdown (:297-313): in P0 of the next
// tick the member's own record becomes DEAD inc+1 and is spread; when that gossip is swept at the member, it stops
int swim_leave(swim_handle* h, uint32_t m) {
  GROUP_ALL(swim_leave(s, m));
  if (!h || m >= h->d.N) return SWIM_EINVAL;
  if (h->d.implicit) return SWIM_EUNSUPPORTED;  // implicit views: the tables are not stored
  HIPCK(hipStreamSynchronize(h->stream));
  uint32_t dt = 0, req = 0;
  HIPCK(hipMemcpy(&dt, h->d.dead_tick + m, 4, hipMemcpyDeviceToHost));
  if (dt != NEVER) return SWIM_EINVAL;
  const uint32_t one = 1;  // every shard: k_gossip_apply keeps ALIVE receipts about a leaver (its DEAD may arrive in P1)
  HIPCK(h2d(h->stream, h->d.leaving + m, &one, 4));
  if (!owns(h, m)) return SWIM_OK;
  HIPCK(hipMemcpy(&req, h->d.pending_inc + m, 4, hipMemcpyDeviceToHost));
  req |= 2u;
  HIPCK(h2d(h->stream, h->d.pending_inc + m, &req, 4));
  return SWIM_OK;
}

int swim_set_member_config(swim_handle* h, uint32_t m, const swim_member_config* mc) {
  GROUP_ALL(swim_set_member_config(s, m, mc));
  if (!h || !mc || m >= h->d.N) return SWIM_EINVAL;
  Dev& d = h->d;
  const bool dormant = m >= d.N - d.n_dormant && (h->joined.empty() || !h->joined[m]);
  if (h->tick > 0 && !dormant) return SWIM_EINVAL;  // a running member's ClusterConfig is fixed
  uint32_t pt = 0, tt = 0;
  if (mc->ping_timeout_ms >= mc->ping_interval_ms || mc->ping_req_members > 8 ||
      !to_ticks(mc->ping_interval_ms, h->cfg.tick_ms, &pt) || !to_ticks(mc->ping_timeout_ms, h->cfg.tick_ms, &tt) || pt == 0)
    return SWIM_EINVAL;
  const uint32_t v[4] = {pt, tt, mc->ping_req_members, mc->sync_group};
  HIPCK(hipStreamSynchronize(h->stream));
  HIPCK(h2d(h->stream, d.mcfg + 4ull * m, v, sizeof(v)));
  if (h->cfg.init_mode == SWIM_INIT_PRECONVERGED && d.mode != SWIM_MODE_RUMOR) {
    // the PRECONVERGED schedule phase under the member's own interval (k_init_members, SEMANTICS.md §3)
    const uint32_t np = 1u + philox(m, 1, 0, 0, d.seed_lo ^ SALT_INIT, d.seed_hi).x % pt;
    HIPCK(h2d(h->stream, d.nextPing + m, &np, 4));
  } else if (h->cfg.init_mode == SWIM_INIT_COLD_JOIN && !dormant) {
    // an initial member starts at tick 0 (start0): its first ping follows its own pingInterval (a dormant member's
    // is set by k_join at its start tick)
    HIPCK(h2d(h->stream, d.nextPing + m, &pt, 4));
  }
  if (!d.permember) {  // the kernels read mcfg from now on (Dev is passed by value and through d.self)
    d.permember = 1;
    HIPCK(h2d(h->stream, (void*)d.self, &d, sizeof(Dev)));
  }
  return SWIM_OK;
}

int swim_set_default_loss(swim_handle* h, uint32_t pct) {
  GROUP_ALL(swim_set_default_loss(s, pct));
  if (!h || pct > 100) return SWIM_EINVAL;
  h->loss = pct;
  return push_epoch(h);
}

int swim_set_partition(swim_handle* h, const uint32_t* g) {
  GROUP_ALL(swim_set_partition(s, g));
  if (!h) return SWIM_EINVAL;
  if (g) {
    h->group.assign(g, g + h->d.N);
    h->partitioned = true;
    // block() writes DEAD_LINK_SETTINGS over a custom setting of every cross-group link (NetworkEmulator.java:141-150)
    std::vector<uint64_t> drop;
    for (const auto& kv : h->link_cur) {
      uint32_t src = (uint32_t)((kv.first - 1) >> 32), dst = (uint32_t)(kv.first - 1);
      if (g[src] != g[dst]) drop.push_back(kv.first);
    }
    for (uint64_t key : drop) link_change(h, key, LK_NONE);
    if (!drop.empty()) {
      int rc = upload_links(h);
      if (rc) return rc;
    }
  } else {
    h->partitioned = false;
  }
  return push_epoch(h);
}

int swim_unblock_all(swim_handle* h) {  // NetworkEmulator.unblockAll: customLinkSettings.clear() (:186-192)
  GROUP_ALL(swim_unblock_all(s));
  if (!h) return SWIM_EINVAL;
  h->partitioned = false;
  if (!h->link_cur.empty()) {
    std::vector<uint64_t> keys;
    for (const auto& kv : h->link_cur) keys.push_back(kv.first);
    for (uint64_t key : keys) link_change(h, key, LK_NONE);
    int rc = upload_links(h);
    if (rc) return rc;
  }
  return push_epoch(h);
}

int swim_set_link_loss(swim_handle* h, uint32_t src, uint32_t dst, uint32_t pct) {
  GROUP_ALL(swim_set_link_loss(s, src, dst, pct));
  if (!h || src >= h->d.N || dst >= h->d.N || pct > 100) return SWIM_EINVAL;
  link_change(h, link_key_of(src, dst), pct);
  return upload_links(h);
}

// the delay index of a mean delay (0: none, or a delay that never reaches a tick); registers its threshold table
static int delay_index(swim_handle* h, uint32_t delay_ms, uint32_t* idx) {
  std::vector<uint32_t> t;
  if (!delay_table(delay_ms, h->cfg.tick_ms, &t)) return fail(h, SWIM_EINVAL, "mean delay above 11 x tick_ms");
  *idx = 0;
  if (t.empty()) return SWIM_OK;  // no message can be delayed past its tick
  if (t.size() > h->d.EMAX) return fail(h, SWIM_EUNSUPPORTED, "mean delay above swim_config.delay_cap_ms");
  for (uint32_t i = 1; i < (uint32_t)h->delays.size(); ++i)
    if (h->delays[i] == delay_ms) {
      *idx = i;
      return SWIM_OK;
    }
  if (h->delays.size() >= DTAB) return fail(h, SWIM_ECAPACITY, "more than 15 distinct mean delays");
  *idx = (uint32_t)h->delays.size();
  h->delays.push_back(delay_ms);
  const uint32_t len = (uint32_t)t.size();
  HIPCK(h2d(h->stream, h->d.dly_thr + (size_t)*idx * 256, t.data(), 4ull * len));
  HIPCK(h2d(h->stream, h->d.dly_len + *idx, &len, 4));
  if (!h->d.dly_on) {  // from now on the gossip plane queues delayed receipts and SYNC messages are stored
    h->d.dly_on = 1;
    HIPCK(h2d(h->stream, (void*)h->d.self, &h->d, sizeof(Dev)));
  }
  return SWIM_OK;
}

int swim_set_default_link_settings(swim_handle* h, uint32_t pct, uint32_t delay_ms) {
  GROUP_ALL(swim_set_default_link_settings(s, pct, delay_ms));
  if (!h || pct > 100) return SWIM_EINVAL;
  uint32_t idx;
  int rc = delay_index(h, delay_ms, &idx);
  if (rc) return rc;
  h->delay_idx = idx;
  return swim_set_default_loss(h, pct);  // a new settings epoch with both
}

int swim_set_link_settings(swim_handle* h, uint32_t src, uint32_t dst, uint32_t pct, uint32_t delay_ms) {
  GROUP_ALL(swim_set_link_settings(s, src, dst, pct, delay_ms));
  if (!h || src >= h->d.N || dst >= h->d.N || pct > 100) return SWIM_EINVAL;
  uint32_t idx;
  int rc = delay_index(h, delay_ms, &idx);
  if (rc) return rc;
  link_change(h, link_key_of(src, dst), pct | (idx << 8));
  return upload_links(h);
}

int swim_emulator_counters(swim_handle* h, uint64_t* out, size_t cap) {
  if (!h || !out || cap < 2ull * h->cfg.n_members) return SWIM_EINVAL;
  if (h->grp) {  // each shard counted the sends it evaluated (its issuers' FD / SYNC / metadata, its targets' gossip)
    std::vector<uint64_t> part(2ull * h->cfg.n_members);
    std::fill(out, out + part.size(), 0ull);
    return group_all(h, [&](swim_handle* s) {
      const int rc = swim_emulator_counters(s, part.data(), part.size());
      for (size_t i = 0; rc == SWIM_OK && i < part.size(); ++i) out[i] += part[i];
      return rc;
    });
  }
  if (!h->d.em) return fail(h, SWIM_EUNSUPPORTED, "emulator counters need SWIM_FLAG_EMULATOR_COUNTERS");
  HIPCK(hipStreamSynchronize(h->stream));
  HIPCK(hipMemcpy(out, h->d.em, 16ull * h->d.N, hipMemcpyDeviceToHost));
  return SWIM_OK;
}

int swim_unblock_link(swim_handle* h, uint32_t src, uint32_t dst) {
  GROUP_ALL(swim_unblock_link(s, src, dst));
  if (!h || src >= h->d.N || dst >= h->d.N) return SWIM_EINVAL;
  if (!h->link_cur.count(link_key_of(src, dst))) return SWIM_OK;
  link_change(h, link_key_of(src, dst), LK_NONE);
  return upload_links(h);
}

int swim_current_tick(swim_handle* h, uint64_t* t) {
  if (!h || !t) return SWIM_EINVAL;
  *t = h->tick;
  return SWIM_OK;
}

int swim_read_row(swim_handle* h, uint32_t obs, uint64_t* out, size_t cap) {
  GROUP_OWNER(obs, swim_read_row(s, obs, out, cap));
  if (!h || obs >= h->d.N || cap < h->d.N || !owns(h, obs)) return SWIM_EINVAL;
  HIPCK(hipStreamSynchronize(h->stream));
  if (h->d.implicit) {  // RUMOR mode: every row is the PRECONVERGED row
    for (uint32_t s = 0; s < h->d.N; ++s) out[s] = PRE_REC;
    return SWIM_OK;
  }
  std::vector<uint32_t> k(h->d.N), a(h->d.N);  // the two planes, joined into logical records (swim_common.h)
  HIPCK(hipMemcpy(k.data(), h->d.rowk + lidx(h->d, obs) * h->d.NS, 4ull * h->d.N, hipMemcpyDeviceToHost));
  HIPCK(hipMemcpy(a.data(), h->d.rowa + lidx(h->d, obs) * h->d.NS, 4ull * h->d.N, hipMemcpyDeviceToHost));
  for (uint32_t s = 0; s < h->d.N; ++s) out[s] = (k[s] & 3u) == ST_ABSENT ? 0 : rec_join(k[s], a[s]);
  return SWIM_OK;
}

int swim_export_sync_frame(swim_handle* h, uint32_t obs, uint32_t kind, uint8_t* buf, size_t cap, size_t* len) {
  if (!h || !len) return SWIM_EINVAL;
  std::vector<uint64_t> row(h->d.N);
  int rc = swim_read_row(h, obs, row.data(), row.size());
  if (rc != SWIM_OK) return rc;
  std::vector<swim_wire_record> recs;  // prepareSyncDataMsg (MembershipProtocolImpl.java:446-454): the whole table
  for (uint32_t s = 0; s < h->d.N; ++s)
    if (rec_status(row[s]) != ST_ABSENT) recs.push_back(swim_wire_record{s, rec_status(row[s]), rec_inc(row[s])});
  return swim_wire_sync_frame(kind, obs, nullptr, "default", recs.data(), recs.size(), buf, cap, len);
}

int swim_state_hash(swim_handle* h, uint64_t* out, size_t cap) {
  if (!h || cap < 6ull * h->d.N) return SWIM_EINVAL;
  if (h->grp) {  // each shard fills its observers' words and leaves the others zero
    std::vector<uint64_t> part(6ull * h->d.N);
    std::fill(out, out + 6ull * h->d.N, 0ull);
    const bool slots = h->grp->slots;
    bool first = true;
    return group_all(h, [&](swim_handle* s) {
      const int rc = swim_state_hash(s, part.data(), part.size());
      // slot-sharded: row, lists and scalars are replicated (taken once); the event and held-gossip words are
      // sums over each shard's own gossips (SEMANTICS.md §9)
      for (size_t i = 0; rc == SWIM_OK && i < part.size(); ++i)
        if (!slots || first || i % 6 == 3 || i % 6 == 4) out[i] += part[i];
      first = false;
      return rc;
    });
  }
  uint64_t* dout = nullptr;
  HIPCK(hipMalloc(&dout, 48ull * h->d.N));
  HIPCK(hipMemsetAsync(dout, 0, 48ull * h->d.N, h->stream));  // other shards' observers stay zero
  launch_hash(h->d, dout, (uint32_t)h->tick, h->stream);
  HIPCK(hipStreamSynchronize(h->stream));
  HIPCK(hipMemcpy(out, dout, 48ull * h->d.N, hipMemcpyDeviceToHost));
  hipFree(dout);
  return check_err(h);
}

int swim_read_lists(swim_handle* h, uint32_t obs, uint32_t* fd, uint32_t* fd_len, uint32_t* gl, uint32_t* g_len,
                    size_t cap, int32_t* cursors) {
  GROUP_OWNER(obs, swim_read_lists(s, obs, fd, fd_len, gl, g_len, cap, cursors));
  if (!h || obs >= h->d.N || !owns(h, obs)) return SWIM_EINVAL;
  HIPCK(hipStreamSynchronize(h->stream));
  uint32_t fl = 0, glen = 0;
  MS ms;
  HIPCK(hipMemcpy(&ms, h->d.ms + obs, sizeof(MS), hipMemcpyDeviceToHost));
  fl = ms.fdLen;
  glen = ms.gLen;
  if (fl > cap || glen > cap) return SWIM_EINVAL;
  if (h->d.implicit) {  // RUMOR mode: the PRECONVERGED permutations (list_at)
    const FeistelPerm P0 = list_perm(h->d, obs, 0), P1 = list_perm(h->d, obs, 1);
    for (uint32_t p = 0; p < fl; ++p) fd[p] = list_at(P0, obs, p);
    for (uint32_t p = 0; p < glen; ++p) gl[p] = list_at(P1, obs, p);
  } else {
    HIPCK(hipMemcpy(fd, h->d.fdl + lidx(h->d, obs) * h->d.LCAP, 4ull * fl, hipMemcpyDeviceToHost));
    HIPCK(hipMemcpy(gl, h->d.gl + lidx(h->d, obs) * h->d.LCAP, 4ull * glen, hipMemcpyDeviceToHost));
  }
  cursors[0] = ms.pingIdx;
  cursors[1] = ms.remoteIdx;
  *fd_len = fl;
  *g_len = glen;
  return SWIM_OK;
}

int swim_read_gossips(swim_handle* h, uint32_t obs, uint64_t* ids, uint32_t* inf, size_t cap, size_t* n_out) {
  if (h && h->grp && h->grp->slots) {  // slot-sharded: the union of every shard's own gossips, in id order
    if (!n_out || obs >= h->d.N) return SWIM_EINVAL;
    std::vector<std::pair<uint64_t, uint32_t>> all;
    std::vector<uint64_t> i2(cap);
    std::vector<uint32_t> f2(cap);
    const int rc = group_all(h, [&](swim_handle* s) {
      size_t n = 0;
      const int r = swim_read_gossips(s, obs, i2.data(), f2.data(), cap, &n);
      for (size_t i = 0; r == SWIM_OK && i < n; ++i) all.emplace_back(i2[i], f2[i]);
      return r;
    });
    if (rc != SWIM_OK) return rc;
    std::sort(all.begin(), all.end());
    if (all.size() > cap) return SWIM_ECAPACITY;
    for (size_t i = 0; i < all.size(); ++i) ids[i] = all[i].first, inf[i] = all[i].second;
    *n_out = all.size();
    return SWIM_OK;
  }
  GROUP_OWNER(obs, swim_read_gossips(s, obs, ids, inf, cap, n_out));
  if (!h || obs >= h->d.N || !n_out || !owns(h, obs)) return SWIM_EINVAL;
  HIPCK(hipStreamSynchronize(h->stream));
  const Dev& d = h->d;
  std::vector<uint32_t> used(d.SLOTS), born(d.SLOTS);
  std::vector<uint16_t> col(d.SLOTS);
  std::vector<uint64_t> gid(d.SLOTS);
  HIPCK(hipMemcpy(used.data(), d.slot_used, 4ull * d.SLOTS, hipMemcpyDeviceToHost));
  HIPCK(hipMemcpy(gid.data(), d.slot_gid, 8ull * d.SLOTS, hipMemcpyDeviceToHost));
  HIPCK(hipMemcpy(born.data(), d.slot_ctick, 4ull * d.SLOTS, hipMemcpyDeviceToHost));
  HIPCK(hipMemcpy(col.data(), d.S + (size_t)obs * d.SLOTS, 2ull * d.SLOTS, hipMemcpyDeviceToHost));  // member-major
  uint32_t first = 0, dt = 0;
  HIPCK(hipMemcpy(&first, d.firstGossip + obs, 4, hipMemcpyDeviceToHost));
  HIPCK(hipMemcpy(&dt, d.dead_tick + obs, 4, hipMemcpyDeviceToHost));
  if (dt != NEVER) {  // a crashed member keeps no gossips (its entries stay only for the infectedFrom replay)
    *n_out = 0;
    return SWIM_OK;
  }
  std::vector<std::pair<uint64_t, uint32_t>> out;
  for (uint32_t g = 0; g < d.SLOTS; ++g) {
    const uint16_t e = col[g];
    if (!used[g] || !(e & S16_EVER) || (e & S16_SWEPT)) continue;
    const uint32_t c = s16_tick(e, (uint32_t)h->tick + d.lat);
    if (c < born[g]) continue;   // an earlier gossip of the recycled slot (s_get)
    if (c >= h->tick) continue;  // receipt of the next tick's P4
    uint32_t rb = (first == NEVER || c <= first) ? 0 : (c - first + d.gossip_t - 1) / d.gossip_t;
    out.emplace_back(gid[g], rb);
  }
  std::sort(out.begin(), out.end());
  if (out.size() > cap) return SWIM_ECAPACITY;
  for (size_t i = 0; i < out.size(); ++i) {
    ids[i] = out[i].first;
    inf[i] = out[i].second;
  }
  *n_out = out.size();
  return SWIM_OK;
}

int swim_drain_events(swim_handle* h, swim_event* out, size_t cap, size_t* n_out) {
  if (!h || !n_out) return SWIM_EINVAL;
  if (h->grp) {  // every shard's events, merged in (tick, observer, seq) order
    auto& ev = h->grp->events;
    // events left over from an earlier call (cap smaller than what was buffered) are already sorted and numbered;
    // only this call's events, all of later ticks, are sorted and numbered here
    const size_t old = ev.size();
    std::vector<swim_event> buf(65536);
    const int rc = group_all(h, [&](swim_handle* s) {
      size_t n = 0;
      do {
        const int r = swim_drain_events(s, buf.data(), buf.size(), &n);
        if (r != SWIM_OK) return r;
        ev.insert(ev.end(), buf.begin(), buf.begin() + (long)n);
      } while (n == buf.size());
      return SWIM_OK;
    });
    if (rc != SWIM_OK) return rc;
    if (h->grp->slots) {  // one observer's events of a tick come from several shards: P4's gossip-id order, renumbered
      std::stable_sort(ev.begin() + (long)old, ev.end(), [](const swim_event& a, const swim_event& b) {
        if (a.tick != b.tick) return a.tick < b.tick;
        if (a.observer != b.observer) return a.observer < b.observer;
        return a.subject != b.subject ? a.subject < b.subject : a.pad < b.pad;
      });
      for (size_t i = old; i < ev.size(); ++i) ev[i].seq = h->grp->evcount[ev[i].observer]++;
    } else {
      std::stable_sort(ev.begin() + (long)old, ev.end(), [](const swim_event& a, const swim_event& b) {
        if (a.tick != b.tick) return a.tick < b.tick;
        if (a.observer != b.observer) return a.observer < b.observer;
        return a.seq < b.seq;
      });
    }
    const size_t k = std::min(cap, ev.size());
    std::copy(ev.begin(), ev.begin() + (long)k, out);
    ev.erase(ev.begin(), ev.begin() + (long)k);
    *n_out = k;
    return SWIM_OK;
  }
  HIPCK(hipStreamSynchronize(h->stream));
  uint32_t n = 0;
  HIPCK(hipMemcpy(&n, h->d.ev_n, 4, hipMemcpyDeviceToHost));
  n = std::min(n, h->d.EVCAP);
  if (n) {
    size_t base = h->host_events.size();
    h->host_events.resize(base + n);
    HIPCK(hipMemcpy(h->host_events.data() + base, h->d.ev, sizeof(swim_event) * n, hipMemcpyDeviceToHost));
    HIPCK(hipMemsetAsync(h->d.ev_n, 0, 4, h->stream));
  }
  auto& ev = h->host_events;
  std::stable_sort(ev.begin(), ev.end(), [](const swim_event& a, const swim_event& b) {
    if (a.tick != b.tick) return a.tick < b.tick;
    if (a.observer != b.observer) return a.observer < b.observer;
    return a.seq < b.seq;
  });
  size_t k = std::min(cap, ev.size());
  std::copy(ev.begin(), ev.begin() + (long)k, out);
  ev.erase(ev.begin(), ev.begin() + (long)k);
  *n_out = k;
  return SWIM_OK;
}

int swim_counters_get(swim_handle* h, swim_counters* out) {
  if (!h || !out) return SWIM_EINVAL;
  if (h->grp) {  // the shards' shares summed (the tick is common)
    swim_counters sum{}, c{};
    const int rc = group_all(h, [&](swim_handle* s) {
      const int r = swim_counters_get(s, &c);
      const uint64_t* a = (const uint64_t*)&c;
      uint64_t* t = (uint64_t*)&sum;
      for (size_t i = 1; r == SWIM_OK && i < sizeof(c) / 8; ++i) t[i] += a[i];
      sum.tick = c.tick;
      return r;
    });
    *out = sum;
    return rc;
  }
  HIPCK(hipStreamSynchronize(h->stream));
  unsigned long long c[C_NCTR];
  HIPCK(hipMemcpy(c, h->d.ctr, sizeof(c), hipMemcpyDeviceToHost));
  {  // the member kernel's rows of counters 0-7
    std::vector<unsigned long long> sh((size_t)CSH * CSTRIDE);
    HIPCK(hipMemcpy(sh.data(), h->d.ctr_sh, 8 * sh.size(), hipMemcpyDeviceToHost));
    for (uint32_t r = 0; r < CSH; ++r)
      for (uint32_t i = 0; i < 8; ++i) c[i] += sh[(size_t)r * CSTRIDE + i];
  }
  std::memset(out, 0, sizeof(*out));
  out->tick = h->tick;
  out->record_compares = c[C_R];
  out->row_writes = c[C_W];
  out->messages = c[C_M];
  out->gossip_messages = c[C_G];
  out->events = c[C_E];
  out->messages_lost = c[C_LOST];
  out->gossips_created = c[C_GCREATED];
  out->sync_merges = c[C_SYNCMERGE];
  out->device_bytes = h->bytes;
  out->diff_ns = (uint64_t)(h->prof_ms[0] * 1e6);
  out->member_ns = (uint64_t)(h->prof_ms[1] * 1e6);
  out->gossip_ns = (uint64_t)(h->prof_ms[2] * 1e6);
  out->diff_launches = h->prof_diff_launches;
  out->diff_msgs = c[C_DIFFMSG];
  out->ack_resolved = c[C_ACKRES];
  out->ack_resolved_total = c[C_ACKRES_ALL];
  out->diff_msgs_total = c[C_DIFFMSG_ALL];
  // the payloads streamed from the 8-bit shadow plane compared 2 B per subject, the others (C_DIFFWIDE) 8 B
  const uint64_t nsub = h->d.N;
  out->diff_key_bytes = nsub * (2 * (c[C_DIFFMSG] - std::min(c[C_DIFFMSG], c[C_DIFFWIDE])) + 8 * c[C_DIFFWIDE]);
  out->diff_key_bytes_total =
      nsub * (2 * (c[C_DIFFMSG_ALL] - std::min(c[C_DIFFMSG_ALL], c[C_DIFFWIDE_ALL])) + 8 * c[C_DIFFWIDE_ALL]);
  out->exchange_ns = (uint64_t)(h->xchg_ms * 1e6);
  return SWIM_OK;
}

const char* swim_last_error(swim_handle* h) { return h ? h->err.c_str() : "null handle"; }

int swim_debug_fallbacks(swim_handle* h, uint64_t* out, size_t n) {
  if (!h || !out || n > FB_N) return SWIM_EINVAL;
  std::fill(out, out + n, 0ull);
  if (h->grp) {  // summed over the shards
    std::vector<uint64_t> part(n);
    return group_all(h, [&](swim_handle* s) {
      const int rc = swim_debug_fallbacks(s, part.data(), n);
      for (size_t i = 0; rc == SWIM_OK && i < n; ++i) out[i] += part[i];
      return rc;
    });
  }
  if (!h->d.fb) return SWIM_EUNSUPPORTED;  // not counted (SWIM_CAPS / SWIM_FALLBACKS unset at create)
  HIPCK(hipStreamSynchronize(h->stream));
  HIPCK(hipMemcpy(out, h->d.fb, 8 * n, hipMemcpyDeviceToHost));
  return SWIM_OK;
}

int swim_debug_caps(swim_handle* h, uint64_t* out, size_t n) {
  if (!h || !out || n > 8) return SWIM_EINVAL;
  if (h->grp) return SWIM_EUNSUPPORTED;
  const uint64_t v[8] = {h->d.SPR, h->d.BCAP, h->d.RCAP, h->d.RPCAP, h->d.HCAP, h->growths, 0, 0};
  for (size_t i = 0; i < n; ++i) out[i] = v[i];
  return SWIM_OK;
}

int swim_debug_holders(swim_handle* h, uint32_t first, uint32_t n, uint32_t* out) {
  if (!h || !out) return SWIM_EINVAL;
  if (h->grp) return SWIM_EUNSUPPORTED;
  const Dev& d = h->d;
  if (d.W > 1 || (uint64_t)first + n > d.N) return d.W > 1 ? SWIM_EUNSUPPORTED : SWIM_EINVAL;
  if (n == 0) return SWIM_OK;
  uint32_t* buf = nullptr;
  HIPCK(hipMalloc(&buf, 20ull * n));
  launch_dbg_holders(d, first, n, buf, h->stream);
  HIPCK(hipStreamSynchronize(h->stream));
  const hipError_t e = hipMemcpy(out, buf, 20ull * n, hipMemcpyDeviceToHost);
  hipFree(buf);
  HIPCK(e);
  return SWIM_OK;
}

int swim_debug_set_incarnation(swim_handle* h, uint32_t m, uint32_t inc) {
  if (!h) return SWIM_EINVAL;
  if (h->grp || h->d.W > 1) return SWIM_EUNSUPPORTED;
  const Dev& d = h->d;
  if (m >= d.N || d.implicit) return SWIM_EINVAL;
  if (inc >= INC_LIMIT) return SWIM_ECAPACITY;
  HIPCK(hipStreamSynchronize(h->stream));
  if (h->tick > 0) {  // a SYNC / SYNC_ACK of m still in flight carries m's live row: the host write would reach it
    const uint32_t b = (uint32_t)((h->tick - 1) & 1);
    uint32_t nm = 0;
    HIPCK(hipMemcpy(&nm, d.nmsg + b, 4, hipMemcpyDeviceToHost));
    nm = std::min(nm, d.MSGCAP);
    std::vector<SyncMsg> v(nm);
    if (nm) HIPCK(hipMemcpy(v.data(), d.msgs[b], nm * sizeof(SyncMsg), hipMemcpyDeviceToHost));
    for (const SyncMsg& q : v)
      if (q.src == m && q.payload == NEVER && !(q.kind & KF_DEFER)) {
        h->err = "swim_debug_set_incarnation: member " + std::to_string(m) + " has a live-row payload in flight";
        return SWIM_EINVAL;
      }
  }
  uint32_t* w = d.rowk + lidx(d, m) * d.NS + m;
  uint32_t k = 0;
  HIPCK(hipMemcpy(&k, w, 4, hipMemcpyDeviceToHost));
  k = (inc << 2) | (k & 3u);
  HIPCK(hipMemcpy(w, &k, 4, hipMemcpyHostToDevice));
  if (d.rowk8) {
    const uint8_t k8 = key8(k);
    HIPCK(hipMemcpy(d.rowk8 + lidx(d, m) * d.NS8 + m, &k8, 1, hipMemcpyHostToDevice));
  }
  return SWIM_OK;
}

// debugging aid (not part of the ABI header): the gossip send log of SWIM_SEND_LOG (tick, sender, gid lo/hi, target)
int swimdbg_send_log(swim_handle* h, uint32_t* out, size_t cap, size_t* n) {
  if (!h || !h->d.dbg_send) return SWIM_EINVAL;
  HIPCK(hipStreamSynchronize(h->stream));
  uint32_t cnt = 0;
  HIPCK(hipMemcpy(&cnt, h->d.dbg_send_n, 4, hipMemcpyDeviceToHost));
  cnt = std::min<uint32_t>(cnt, h->d.dbg_send_cap);
  cnt = (uint32_t)std::min<size_t>(cnt, cap);
  HIPCK(hipMemcpy(out, h->d.dbg_send, 20ull * cnt, hipMemcpyDeviceToHost));
  *n = cnt;
  return SWIM_OK;
}

// debugging aid (not part of the ABI header): the scalar fields folded into the "misc" state-hash word
int swimdbg_scalars(swim_handle* h, uint32_t m, uint64_t* out) {
  if (!h || !owns(h, m)) return SWIM_EINVAL;
  HIPCK(hipStreamSynchronize(h->stream));
  MS ms;
  uint32_t ns = 0;
  HIPCK(hipMemcpy(&ms, h->d.ms + m, sizeof(MS), hipMemcpyDeviceToHost));
  HIPCK(hipMemcpy(&ns, h->d.nextSync + m, 4, hipMemcpyDeviceToHost));
  const uint32_t v[6] = {ms.cidCnt, ms.syncSeq, ms.gCounter, ns, ms.fdPeriod, ms.gPeriod};
  for (int i = 0; i < 6; ++i) out[i] = (i == 3 && v[i] == NEVER) ? ~0ull : v[i];
  return SWIM_OK;
}

// debugging aid (not part of the ABI header): one member's gossip-round ring: [tick, spread, cnt, targets...] x LOGW
int swimdbg_read_log(swim_handle* h, uint32_t m, uint32_t* out, size_t cap, uint32_t* logw, uint32_t* fanout,
                     uint32_t* pos) {
  const Dev& d = h->d;
  size_t need = (size_t)d.LOGW * (3 + d.F);
  if (cap < need) return SWIM_EINVAL;
  HIPCK(hipStreamSynchronize(h->stream));
  std::vector<uint32_t> t(d.LOGW), sp(d.LOGW), c(d.LOGW), tg((size_t)d.LOGW * d.F);
  HIPCK(hipMemcpy(t.data(), d.log_tick + (size_t)m * d.LOGW, 4ull * d.LOGW, hipMemcpyDeviceToHost));
  HIPCK(hipMemcpy(sp.data(), d.log_spread + (size_t)m * d.LOGW, 4ull * d.LOGW, hipMemcpyDeviceToHost));
  HIPCK(hipMemcpy(c.data(), d.log_cnt + (size_t)m * d.LOGW, 4ull * d.LOGW, hipMemcpyDeviceToHost));
  HIPCK(hipMemcpy(tg.data(), d.log_tg + (size_t)m * d.LOGW * d.F, 4ull * d.LOGW * d.F, hipMemcpyDeviceToHost));
  HIPCK(hipMemcpy(pos, d.log_pos + m, 4, hipMemcpyDeviceToHost));
  for (uint32_t e = 0; e < d.LOGW; ++e) {
    uint32_t* o = out + (size_t)e * (3 + d.F);
    o[0] = t[e];
    o[1] = sp[e];
    o[2] = c[e];
    for (uint32_t i = 0; i < d.F; ++i) o[3 + i] = tg[(size_t)e * d.F + i];
  }
  *logw = d.LOGW;
  *fanout = d.F;
  return SWIM_OK;
}

}  // extern "C"
