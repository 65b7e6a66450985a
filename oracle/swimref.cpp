// oracle/swimref.cpp — TEST INFRASTRUCTURE. CPU restatement of the reference's SWIM hot path.
//
// This is the oracle, not the product. Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg load
// liboracle_swimref.so, and only as the checker or the timed CPU baseline. It exports the same C ABI as
// libswimhip (include/swimhip.h), so a parity test can drive both backends through one interface.
//
// Shape: one Member object per simulated member. Each holds the fields of FailureDetectorImpl,
// GossipProtocolImpl, MembershipProtocolImpl and MetadataStoreImpl. Members talk only through explicit Msg
// objects on an in-memory transport. Loss is applied at the sender, and a failed send errors the caller at once
// (TransportImpl.java:205-232, NetworkEmulator.java:231-248). requestResponse is a subscription keyed by the
// correlation id. Gossip keeps real infectedFrom sets. Concurrency and timing follow SEMANTICS.md. Every method
// cites the Java it restates. Paths are relative to
// /root/reference/cluster/src/main/java/io/scalecube/cluster/ unless they start with transport/.
//
// Parity pin: the reference is Java 8 + Reactor, with no JDK, Maven or jars in this image, so it cannot
// run here. isOverrides is pinned by MembershipRecordTest.java:34-108 (tests/test_oracle_known_answers.py). ClusterMath
// is pinned by its closed forms. Event ordering and timing are pinned only by SEMANTICS.md, which makes parity for
// them "spec-pinned", not reference-pinned.
#include <algorithm>
#include <cmath>
#include <atomic>
#include <condition_variable>
#include <functional>
#include <mutex>
#include <thread>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <map>
#include <memory>
#include <set>
#include <string>
#include <vector>

#include "../include/swimhip.h"
#include "../include/swimhip_selftest.h"
#include "rng.h"

using namespace swimref;

namespace {

constexpr uint32_t NONE = 0xFFFFFFFFu;
constexpr uint64_t NEVER = ~0ull;
constexpr uint32_t USER_SUBJ = 0xFFFFFFFFu;  // gossip subject of a user gossip (no membership record)

enum St : uint8_t { ABSENT = 0, ALIVE = 1, SUSPECT = 2, DEAD = 3 };  // MemberStatus.java:6-15 (+absent)
enum Kind : uint8_t { K_SYNC = 1, K_SYNC_ACK, K_PING, K_PING_REQ, K_PING_ACK, K_GMD_REQ, K_GMD_RESP, K_GOSSIP };
enum Reason { R_FD, R_GOSSIP, R_SYNC, R_INITIAL, R_TIMEOUT };  // MembershipProtocolImpl.java:54-60
enum Stream { S_FD_SHUFFLE = 1, S_FD_INSERT = 2, S_PINGREQ = 3, S_GOSSIP_SHUFFLE = 4, S_SYNC_PICK = 5 };

struct Rec {
  uint8_t st = ABSENT;
  uint32_t inc = 0;
  bool operator==(const Rec& o) const { return st == o.st && inc == o.inc; }  // MembershipRecord.java:86-99
  bool operator!=(const Rec& o) const { return !(*this == o); }
};

// MembershipRecord.isOverrides (MembershipRecord.java:66-84); r0.st == ABSENT is the `r0 == null` case.
bool is_overrides(Rec r1, Rec r0) {
  if (r0.st == ABSENT) return r1.st == ALIVE;
  if (r0.st == DEAD) return false;
  if (r1.st == DEAD) return true;
  if (r1.inc == r0.inc) return (r1.st != r0.st) && (r1.st == SUSPECT);
  return r1.inc > r0.inc;
}

uint32_t bitlen(uint32_t n) { return n ? 32u - (uint32_t)__builtin_clz(n) : 0u; }  // ClusterMath.java:133-135

using Payload = std::vector<std::pair<uint32_t, Rec>>;

struct Msg {
  uint8_t kind = 0;
  uint32_t src = 0, dst = 0;
  uint32_t cid_iss = NONE, cid_cnt = 0;                  // correlation id (issuer, counter)
  uint32_t pd_from = NONE, pd_to = NONE, pd_orig = NONE;  // PingData (fdetector/PingData.java:6-50)
  uint32_t seq = 0;                                       // syncSeq for SYNC / SYNC_ACK
  uint32_t extra = 0;                                     // delay ticks past lat (NetworkEmulator.tryDelay)
  std::shared_ptr<Payload> payload;                       // SyncData (membership/SyncData.java:11-41)
  uint32_t md_subject = NONE, md_meta = NONE;             // GetMetadataRequest / Response
  uint64_t gid = 0;                                       // gossip id (origin << 32 | counter)
  uint32_t slot = 0;                                      // target slot of a GOSSIP_REQ
  uint32_t g_subj = 0;
  Rec g_rec;                                              // gossip payload: MembershipRecord
  uint64_t g_payload = 0;                                 // user gossip payload (g_subj == USER_SUBJ)
};

struct Sim;

// What one worker produces while it processes its range of members in a tick (SWIMREF_THREADS > 1 splits the members
// into contiguous ranges; the lanes are merged in member order after the tick, so results do not depend on the split)
struct Lane {
  swim_counters ctr;
  std::vector<Msg> out;
  std::vector<swim_event> events;
  std::vector<uint32_t> leaving;
};
thread_local Lane* tl_lane = nullptr;

// a fixed pool of worker threads; the calling thread runs part 0
struct Pool {
  std::vector<std::thread> th;
  std::mutex mu;
  std::condition_variable cv, done;
  std::function<void(int)> job;
  uint64_t gen = 0;
  int pending = 0;
  bool stop = false;
  void start(int n) {
    for (int i = 1; i < n; ++i)
      th.emplace_back([this, i] {
        uint64_t seen = 0;
        for (;;) {
          std::function<void(int)> f;
          {
            std::unique_lock<std::mutex> lk(mu);
            cv.wait(lk, [&] { return stop || gen != seen; });
            if (stop) return;
            seen = gen;
            f = job;
          }
          f(i);
          std::lock_guard<std::mutex> lk(mu);
          if (--pending == 0) done.notify_one();
        }
      });
  }
  void run(const std::function<void(int)>& f) {
    {
      std::lock_guard<std::mutex> lk(mu);
      job = f;
      pending = (int)th.size();
      gen++;
    }
    cv.notify_all();
    f(0);
    std::unique_lock<std::mutex> lk(mu);
    done.wait(lk, [&] { return pending == 0; });
  }
  ~Pool() {
    {
      std::lock_guard<std::mutex> lk(mu);
      stop = true;
    }
    cv.notify_all();
    for (auto& t : th) t.join();
  }
};

struct Member {
  Sim* sim = nullptr;
  uint32_t id = 0;
  bool alive = true;

  // MembershipProtocolImpl state (:82-96) + MetadataStoreImpl.membersMetadata
  std::vector<Rec> table;
  uint32_t tsize = 0;
  std::vector<uint32_t> meta;
  std::map<uint32_t, uint64_t> timers;  // suspicionTimeoutTasks: subject -> deadline tick
  std::vector<uint32_t> seeds;

  // FailureDetectorImpl state (:47-49)
  std::vector<uint32_t> ping;
  int64_t pingIdx = 0;
  uint64_t fdPeriod = 0;
  struct Sub {
    uint32_t cnt;
    int kind;  // 0 DIRECT, 1 PINGREQ
    uint32_t helper, target;
    uint64_t deadline, order;
  };
  std::vector<Sub> subs;  // pending requestResponse subscriptions
  uint64_t subOrder = 0;

  // this member's NetworkEmulator counters (totalMessageSentCount / totalMessageLostCount, NetworkEmulator.java:200-222)
  uint64_t emSent = 0, emLost = 0;

  // GossipProtocolImpl state (:47-53), GossipState.java:8-38
  std::vector<uint32_t> remote;
  int64_t remoteIdx = -1;
  uint64_t gPeriod = 0;
  uint32_t gCounter = 0;
  struct GState {
    uint32_t subj;  // USER_SUBJ: a user gossip (Cluster.spreadGossip) carrying payload
    Rec rec;
    uint64_t payload = 0;
    uint64_t infPeriod;
    // infectedFrom (GossipState.java:8-38) as a sorted vector: the same set semantics in ~4 B per sender (a
    // std::set costs ~40 B per node; C2-shaped runs hold ~10^8 (member, gossip) states with tens of senders each)
    std::vector<uint32_t> infected;
    bool is_infected(uint32_t t) const { return std::binary_search(infected.begin(), infected.end(), t); }
    void add_infected(uint32_t t) {
      auto it = std::lower_bound(infected.begin(), infected.end(), t);
      if (it == infected.end() || *it != t) infected.insert(it, t);
    }
  };
  std::map<uint64_t, GState> gossips;

  // MetadataStoreImpl.fetchMetadata subscriptions (:149-186) + their updateMembership continuation
  struct Fetch {
    uint32_t subj;
    Rec r1;
    int reason;
    bool added;
    uint64_t deadline;
    int group;
  };
  std::map<uint32_t, Fetch> fetches;

  // Mono.whenDelayError over one syncMembership (:456-467); kind 0 = SYNC -> SYNC_ACK, 1 = initial sync
  struct Group {
    int kind;
    uint32_t reply_to, cid_iss, cid_cnt;
    int remaining;
    bool error, sealed;
  };
  std::map<int, Group> groups;
  int nextGroup = 0;

  // start0 (:216-251)
  bool initActive = false, initReceived = false;
  std::set<uint32_t> initCids;
  uint64_t initDeadline = NEVER;

  uint64_t nextPing = NEVER, nextGossip = NEVER, nextSync = NEVER;
  // this member's own FailureDetectorConfig and syncGroup (swim_set_member_config; else the swim_config values)
  uint32_t ping_t = 0, pingTimeout_t = 0, kreq = 0, syncGroup = 0;
  uint32_t pendingInc = 0;  // swim_update_incarnation calls, applied in P0 of the next tick (one bump each)
  bool pendingLeave = false;  // swim_leave (leaveCluster), applied in P0 of the next tick after pendingInc
  uint64_t startTick = NEVER;  // COLD_JOIN: 0 for the initial members, the join tick for a dormant one (swim_join)
  bool dormant = false;
  std::vector<uint64_t> pendingUser;  // swim_spread_gossip payloads, spread in P0 of the next tick before pendingInc
  uint32_t cidCnt = 0, syncSeq = 0, evSeq = 0;
  uint32_t sel[8] = {0};
  uint64_t evHash = 0;

  // ---- helpers implemented below ----
  uint32_t draw(int stream);
  void shuffle(std::vector<uint32_t>& v, int stream);
  void process(uint64_t k, std::vector<Msg>& inbox);
  void start(uint64_t k);
  void send(Msg&& m, uint64_t k, bool gossip = false);
  bool send_sync(uint8_t kind, uint32_t dst, uint32_t cid_iss, uint32_t cid_cnt, uint64_t k);
  void emit_event(uint32_t type, uint32_t subj, uint32_t oldm, uint32_t newm, uint64_t k, uint32_t pad = 0);
  void on_member_event(uint32_t type, uint32_t subj);
  void spread(uint32_t subj, Rec rec, uint64_t payload = 0);
  void update_membership(uint32_t subj, Rec r1, int reason, int group, uint64_t k);
  void finish(int group, bool error, uint64_t k);
  void do_finally(uint32_t subj, Rec r1, int reason);
  void fetch(uint32_t subj, Rec r1, int reason, bool added, int group, uint64_t k);
  void sync_membership(const Payload& p, int reason, int group, uint64_t k);
  const std::vector<Rec>* tickStart = nullptr;  // SWIMREF_DEBUG: the table at the start of P1 (several payloads)
  void complete_group(int g, uint64_t k);
  void on_fd_event(uint32_t target, uint8_t status, uint64_t k);
  void ping_req_step(uint32_t target, uint32_t cnt, uint64_t k);
  void resolve_subs(uint32_t cnt, uint64_t k);
  void do_ping(uint64_t k);
  void do_spread_gossip(uint64_t k);
  void do_sync(uint64_t k);
};

struct Sim {
  FILE* send_log = nullptr;  // debugging aid: SWIMREF_SEND_LOG=<path> lists every counted gossip send
  swim_config cfg;
  uint32_t N = 0;
  uint32_t ping_t = 0, pingTimeout_t = 0, gossip_t = 0, sync_t = 0, syncTimeout_t = 0, md_t = 0, lat = 1;
  uint32_t seed_lo = 0, seed_hi = 0;
  uint64_t tick = 0;
  struct Link {
    uint32_t loss, delay;  // NetworkLinkSettings (NetworkLinkSettings.java:15-38): loss %, mean delay ms
  };
  uint32_t loss = 0, delay = 0;  // defaultLinkSettings (NetworkEmulator.java:113-125)
  bool partitioned = false;
  std::vector<uint32_t> group;
  std::map<uint64_t, Link> custom;  // NetworkEmulator.customLinkSettings: (src << 32 | dst) -> settings
  std::map<uint32_t, std::vector<uint32_t>> dly_thr;  // mean delay ms -> delay thresholds (delay_table)
  std::vector<uint32_t> leaving_done;   // members whose leave completed this tick: stopped from the next tick
  std::vector<Member> members;
  std::vector<uint32_t> md_version;  // each member's own metadata version (GET_METADATA_RESP payload)
  std::vector<std::vector<Msg>> inflight;  // ring indexed by delivery tick % (lat + 256): delays stay below 256 ticks
  std::vector<swim_event> events;
  swim_counters ctr;
  std::string err;
  int threads = 1;  // SWIMREF_THREADS
  // debugging aid (SWIMREF_DEBUG=1): payload records that equal the receiver's start-of-tick row but differ from its
  // live row when a later SYNC / SYNC_ACK of the same tick is merged ([0]), and those of them that override it ([1])
  bool debug = false;
  std::atomic<uint64_t> dbg[4] = {};
  std::vector<uint8_t> leaveRequested;  // SWIMREF_DEBUG: swim_leave was called for the member
  std::vector<Lane> lanes;
  std::unique_ptr<Pool> pool;

  // ClusterMath.suspicionTimeout (ClusterMath.java:123-125) with the member's own pingInterval
  uint32_t suspicion_ticks(uint32_t size, uint32_t member_ping_t) const {
    return cfg.suspicion_mult * bitlen(size) * member_ping_t;
  }
  uint32_t spread_of(uint32_t cluster) const { return cfg.gossip_repeat_mult * bitlen(cluster); }  // :111-113
  uint32_t sweep_of(uint32_t cluster) const { return 2u * (spread_of(cluster) + 1u); }            // :99-102

  // NetworkEmulator.tryFail (transport/.../NetworkEmulator.java:231-248) + NetworkLinkSettings.evaluateLoss (:54-57)
  // getLinkSettings (:57-59): the custom setting of src's emulator for dst, else the default; a partition is the
  // DEAD custom setting on every cross-group link. Returns the loss percent (100 for a dead destination).
  Link link(uint32_t src, uint32_t dst) const {
    if (!custom.empty()) {
      auto it = custom.find(((uint64_t)src << 32) | dst);
      if (it != custom.end()) return it->second;
    }
    if (partitioned && group[src] != group[dst]) return Link{100, 0};  // block(): DEAD_LINK_SETTINGS (:24-26)
    return Link{loss, delay};
  }
  uint32_t link_loss(uint32_t src, uint32_t dst) const {
    if (!members[dst].alive) return 100;
    return link(src, dst).loss;
  }
  // NetworkLinkSettings.evaluateDelay (:64-74): y = -ln(1 - u) * D ms, truncated to ms (longValue) and delivered
  // floor(y / tick_ms) ticks past lat. floor(y / T) >= j  <=>  u >= 1 - exp(-jT/D), so with u = x / 2^32 the extra ticks
  // are the number of thresholds ceil(2^32 (1 - exp(-jT/D))), j = 1.., that x reaches (SEMANTICS.md §2)
  static bool delay_table(uint32_t D, uint32_t T, std::vector<uint32_t>* out) {
    out->clear();
    for (uint32_t j = 1; j <= 256; ++j) {
      const double th = std::ceil((1.0 - std::exp(-(double)j * (double)T / (double)D)) * 4294967296.0);
      if (th > 4294967295.0) return true;
      if (j == 256) return false;  // a delay of 256 ticks or more is reachable: mean delay too long
      out->push_back((uint32_t)th);
    }
    return true;
  }
  uint32_t delay_ticks(uint32_t D, uint32_t x) const {
    const std::vector<uint32_t>& t = dly_thr.at(D);
    return (uint32_t)(std::upper_bound(t.begin(), t.end(), x) - t.begin());
  }
  bool add_delay(uint32_t D) {  // host thread only (settings calls): worker threads only read the tables
    if (D == 0 || dly_thr.count(D)) return true;
    std::vector<uint32_t> t;
    if (!delay_table(D, cfg.tick_ms, &t)) return false;
    dly_thr[D] = std::move(t);
    return true;
  }
  bool lost(uint8_t kind, uint32_t src, uint32_t dst, uint64_t k, uint32_t aux, uint32_t id) const {
    const uint32_t loss = link_loss(src, dst);
    if (loss == 0) return false;
    if (loss >= 100) return true;
    return loss_roll(kind, src, dst, k, aux, id) < loss;
  }
  // NetworkLinkSettings.evaluateLoss (:54-57): nextInt(100) on the message's LOSS_<kind> draw (SEMANTICS.md §2)
  uint32_t loss_roll(uint8_t kind, uint32_t src, uint32_t dst, uint64_t k, uint32_t aux, uint32_t id) const {
    P4 r = philox4x32_10(src, dst, (uint32_t)k, id, seed_lo ^ (SALT_LOSS_BASE + kind), seed_hi ^ (aux * 0x9E3779B9u));
    return next_int(r.v[0], 100);
  }
  // NetworkEmulator.tryFail + tryDelay (NetworkEmulator.java:231-272) of one message src -> dst: -1 if the send
  // fails, else its delay ticks past lat; counts on src's emulator unless the destination refuses the connection
  // (a dead member: TransportImpl.send fails in connect, before the emulator)
  int xmit(uint8_t kind, uint32_t src, uint32_t dst, uint64_t k, uint32_t aux, uint32_t id, Member& em) const;
  int xmit_gossip(uint32_t src, uint32_t dst, uint64_t k, uint32_t slot, uint64_t gid, Member& em) const;
  bool lost_gossip(uint32_t src, uint32_t dst, uint64_t k, uint32_t slot, uint64_t gid) const {
    const uint32_t loss = link_loss(src, dst);
    if (loss == 0) return false;
    if (loss >= 100) return true;
    P4 r = philox4x32_10(src, (uint32_t)k ^ ((slot >> 2) << 31), (uint32_t)(gid >> 32), (uint32_t)gid,
                         seed_lo ^ SALT_LOSS_GOSSIP, seed_hi);
    return next_int(r.v[slot & 3], 100) < loss;
  }
  uint32_t init_draw(uint32_t m, uint32_t what, uint32_t i) const {
    return philox4x32_10(m, what, i, 0, seed_lo ^ SALT_INIT, seed_hi).v[0];
  }
  void run_tick();
};

int Sim::xmit(uint8_t kind, uint32_t src, uint32_t dst, uint64_t k, uint32_t aux, uint32_t id, Member& em) const {
  if (!members[dst].alive) return -1;
  const Link L = link(src, dst);
  em.emSent++;  // tryFail
  if (L.loss >= 100 || (L.loss > 0 && loss_roll(kind, src, dst, k, aux, id) < L.loss)) {
    em.emLost++;
    return -1;
  }
  em.emSent++;  // tryDelay
  if (L.delay == 0) return 0;
  P4 r = philox4x32_10(src, dst, (uint32_t)k, id, seed_lo ^ (SALT_DELAY_BASE + kind), seed_hi ^ (aux * 0x9E3779B9u));
  return (int)delay_ticks(L.delay, r.v[0]);
}
int Sim::xmit_gossip(uint32_t src, uint32_t dst, uint64_t k, uint32_t slot, uint64_t gid, Member& em) const {
  if (!members[dst].alive) return -1;
  const Link L = link(src, dst);
  em.emSent++;
  if (L.loss >= 100 || (L.loss > 0 && lost_gossip(src, dst, k, slot, gid))) {
    em.emLost++;
    return -1;
  }
  em.emSent++;
  if (L.delay == 0) return 0;
  P4 r = philox4x32_10(src, (uint32_t)k ^ ((slot >> 2) << 31), (uint32_t)(gid >> 32), (uint32_t)gid,
                       seed_lo ^ SALT_DELAY_GOSSIP, seed_hi);
  return (int)delay_ticks(L.delay, r.v[slot & 3]);
}

// ---------------------------------------------------------------------------------------------------------------
// selector (SEMANTICS.md §2)
uint32_t Member::draw(int stream) {
  uint32_t c = sel[stream]++;
  return philox4x32_10(id, (uint32_t)stream, c, 0, sim->seed_lo ^ SALT_SEL, sim->seed_hi).v[0];
}
// Collections.shuffle(list, rnd): for i = size..2: swap(i-1, nextInt(i))
void Member::shuffle(std::vector<uint32_t>& v, int stream) {
  for (size_t i = v.size(); i > 1; --i) {
    uint32_t j = next_int(draw(stream), (uint32_t)i);
    std::swap(v[i - 1], v[j]);
  }
}

// transport.send (transport/.../TransportImpl.java:194-202): enqueue for delivery at k + lat
void Member::send(Msg&& m, uint64_t k, bool gossip) {
  (void)gossip;
  Sim& s = *sim;
  (void)s;
  (void)k;
  tl_lane->out.push_back(std::move(m));  // merged into inflight[k + lat + m.extra] after the tick
}

// prepareSyncDataMsg (:446-454) + transport.send; returns false when the send failed
bool Member::send_sync(uint8_t kind, uint32_t dst, uint32_t cid_iss, uint32_t cid_cnt, uint64_t k) {
  Sim& s = *sim;
  uint32_t seq = syncSeq++;
  tl_lane->ctr.messages++;
  const int e = s.xmit(kind, id, dst, k, id, seq, *this);
  if (e < 0) {
    tl_lane->ctr.messages_lost++;
    return false;
  }
  Msg m;
  m.extra = (uint32_t)e;
  m.kind = kind;
  m.src = id;
  m.dst = dst;
  m.cid_iss = cid_iss;
  m.cid_cnt = cid_cnt;
  m.seq = seq;
  auto p = std::make_shared<Payload>();
  p->reserve(tsize);
  for (uint32_t subj = 0; subj < s.N; ++subj)
    if (table[subj].st != ABSENT) p->emplace_back(subj, table[subj]);
  m.payload = std::move(p);
  send(std::move(m), k);
  return true;
}

// sink.next(MembershipEvent) (:548-584) -> user stream, FailureDetectorImpl.onMemberEvent, GossipProtocolImpl.onMemberEvent
// pad: the gossip counter of a GOSSIP event (its id is (subject, pad)). RUMOR mode hashes the events as a sum
// (SEMANTICS.md §9: slot shards each emit a member's events for their own gossips), FULL mode as a chain.
void Member::emit_event(uint32_t type, uint32_t subj, uint32_t oldm, uint32_t newm, uint64_t k, uint32_t pad) {
  Sim& s = *sim;
  uint32_t seq = evSeq++;
  if (s.cfg.mode == SWIM_MODE_RUMOR) {
    evHash += hpair(hpair(((uint64_t)k << 32) | ((uint64_t)type << 30) | subj, ((uint64_t)oldm << 32) | newm), pad);
  } else {
    evHash = hpair(evHash, ((uint64_t)k << 32) | ((uint64_t)type << 30) | subj);
    evHash = hpair(evHash, ((uint64_t)oldm << 32) | newm);
  }
  tl_lane->ctr.events++;
  if (s.cfg.flags & SWIM_FLAG_RECORD_EVENTS) {
    swim_event e{(uint32_t)k, id, seq, type, subj, oldm, newm, pad};
    tl_lane->events.push_back(e);
  }
  on_member_event(type, subj);
}

void Member::on_member_event(uint32_t type, uint32_t subj) {
  // FailureDetectorImpl.onMemberEvent (:321-332)
  if (type == SWIM_EV_REMOVED) {
    auto it = std::find(ping.begin(), ping.end(), subj);
    if (it != ping.end()) ping.erase(it);
  }
  if (type == SWIM_EV_ADDED) {
    size_t sz = ping.size();
    size_t idx = sz > 0 ? next_int(draw(S_FD_INSERT), (uint32_t)sz) : 0;
    ping.insert(ping.begin() + (long)idx, subj);
  }
  // GossipProtocolImpl.onMemberEvent (:185-193)
  if (type == SWIM_EV_REMOVED) {
    auto it = std::find(remote.begin(), remote.end(), subj);
    if (it != remote.end()) remote.erase(it);
  }
  if (type == SWIM_EV_ADDED) remote.push_back(subj);
}

// GossipProtocolImpl.spread -> createAndPutGossip (:124-128,163-169)
void Member::spread(uint32_t subj, Rec rec, uint64_t payload) {
  uint64_t gid = ((uint64_t)id << 32) | gCounter++;
  GState g;
  g.subj = subj;
  g.rec = rec;
  g.payload = payload;
  g.infPeriod = gPeriod;
  gossips.emplace(gid, std::move(g));
  tl_lane->ctr.gossips_created++;
}

// MembershipProtocolImpl.updateMembership (:475-541)
void Member::update_membership(uint32_t subj, Rec r1, int reason, int group, uint64_t k) {
  Sim& s = *sim;
  Rec r0 = table[subj];
  if (!is_overrides(r1, r0)) return;  // :483-485 (completes empty; no doFinally)
  if (subj == id) {                   // :488-509 local member: refute with a higher incarnation
    Rec r2{r0.st, std::max(r0.inc, r1.inc) + 1};
    table[id] = r2;
    tl_lane->ctr.row_writes++;
    spread(id, r2);
    return;
  }
  if (r1.st == DEAD) {  // :512-516
    table[subj] = Rec{};
    tsize--;
  } else {
    if (r0.st == ABSENT) tsize++;
    table[subj] = r1;
  }
  tl_lane->ctr.row_writes++;
  if (r1.st == SUSPECT) {  // :519-523, scheduleSuspicionTimeoutTask (:597-606) computeIfAbsent
    if (!timers.count(subj)) timers[subj] = k + s.suspicion_ticks(tsize, ping_t);
  } else {
    timers.erase(subj);  // cancelSuspicionTimeoutTask (:590-595)
  }
  // emitMembershipEvent (:543-588)
  if (r1.st == DEAD) {
    uint32_t oldm = meta[subj];  // metadataStore.removeMetadata (MetadataStoreImpl.java:135-146)
    meta[subj] = NONE;
    emit_event(SWIM_EV_REMOVED, subj, oldm, NONE, k);
    finish(group, false, k);
    do_finally(subj, r1, reason);
    return;
  }
  if (r0.st == ABSENT && r1.st == ALIVE) {
    fetch(subj, r1, reason, true, group, k);
    return;
  }
  if (r0.st != ABSENT && r0.inc < r1.inc) {
    fetch(subj, r1, reason, false, group, k);
    return;
  }
  finish(group, false, k);
  do_finally(subj, r1, reason);
}

// doFinally of updateMembership (:526-539): spread r1 unless it came from gossip or the initial sync
void Member::do_finally(uint32_t subj, Rec r1, int reason) {
  if (reason != R_GOSSIP && reason != R_INITIAL) spread(subj, r1);
}

// one inner Mono of Mono.whenDelayError terminated (synchronously or later)
void Member::finish(int g, bool error, uint64_t k) {
  if (g < 0) return;
  auto it = groups.find(g);
  if (it == groups.end()) return;
  Group& gr = it->second;
  if (error) gr.error = true;
  if (gr.sealed && gr.remaining == 0) complete_group(g, k);
}

void Member::complete_group(int g, uint64_t k) {
  Group gr = groups[g];
  groups.erase(g);
  if (gr.kind == 0) {
    // onSync doOnSuccess (:351-365): SYNC_ACK with the post-merge table, only if no error
    if (!gr.error) send_sync(K_SYNC_ACK, gr.reply_to, gr.cid_iss, gr.cid_cnt, k);
  } else {
    // start0 doFinally (:244-248): schedulePeriodicSync
    initActive = false;
    nextSync = k + sim->sync_t;
  }
}

// MetadataStoreImpl.fetchMetadata (:149-186)
void Member::fetch(uint32_t subj, Rec r1, int reason, bool added, int group, uint64_t k) {
  Sim& s = *sim;
  uint32_t cnt = cidCnt++;
  tl_lane->ctr.messages++;
  const int e = s.xmit(K_GMD_REQ, id, subj, k, id, cnt, *this);
  if (e < 0) {  // requestResponse send error -> sink.error
    tl_lane->ctr.messages_lost++;
    if (group >= 0) groups[group].error = true;  // error propagates to whenDelayError
    do_finally(subj, r1, reason);
    return;
  }
  Msg m;
  m.extra = (uint32_t)e;
  m.kind = K_GMD_REQ;
  m.src = id;
  m.dst = subj;
  m.cid_iss = id;
  m.cid_cnt = cnt;
  m.md_subject = subj;
  send(std::move(m), k);
  fetches[cnt] = Fetch{subj, r1, reason, added, k + s.md_t, group};
  if (group >= 0) groups[group].remaining++;
}

// syncMembership (:456-467): eager filter of differing records, then sequential updateMembership
void Member::sync_membership(const Payload& p, int reason, int group, uint64_t k) {
  tl_lane->ctr.record_compares += p.size();
  tl_lane->ctr.sync_merges++;
  std::vector<std::pair<uint32_t, Rec>> diff;
  for (auto& e : p)
    if (e.second != table[e.first]) diff.push_back(e);
  if (tickStart)
    for (auto& e : diff)
      if (e.second == (*tickStart)[e.first]) {
        sim->dbg[0]++;
        if (is_overrides(e.second, table[e.first])) sim->dbg[1]++;
      }
  for (auto& e : diff) update_membership(e.first, e.second, reason, group, k);
}

// onFailureDetectorEvent (:370-398)
void Member::on_fd_event(uint32_t target, uint8_t status, uint64_t k) {
  Rec r0 = table[target];
  if (r0.st == ABSENT) return;
  if (r0.st == status) return;
  if (status == ALIVE) {
    send_sync(K_SYNC, target, NONE, 0, k);
  } else {
    tl_lane->ctr.record_compares++;
    update_membership(target, Rec{SUSPECT, r0.inc}, R_FD, -1, k);
  }
}

// doPing error branch (:159-175) + selectPingReqMembers (:349-361) + doPingReq (:178-213)
void Member::ping_req_step(uint32_t target, uint32_t cnt, uint64_t k) {
  Sim& s = *sim;
  std::vector<uint32_t> helpers;
  (void)s;
  if (kreq > 0) {
    std::vector<uint32_t> cand(ping);
    auto it = std::find(cand.begin(), cand.end(), target);
    if (it != cand.end()) cand.erase(it);
    if (!cand.empty()) {
      uint32_t n = (uint32_t)cand.size();
      uint32_t kk = std::min(kreq, n);
      for (uint32_t i = 0; i < kk; ++i) {  // k forward Fisher-Yates steps (SEMANTICS.md §2)
        uint32_t j = i + next_int(draw(S_PINGREQ), n - i);
        std::swap(cand[i], cand[j]);
      }
      helpers.assign(cand.begin(), cand.begin() + kk);
    }
  }
  int timeLeft = (int)ping_t - (int)pingTimeout_t;
  if (timeLeft <= 0 || helpers.empty()) {
    on_fd_event(target, SUSPECT, k);
    return;
  }
  for (uint32_t h : helpers) {
    tl_lane->ctr.messages++;
    const int e = s.xmit(K_PING_REQ, id, h, k, id, cnt, *this);
    if (e < 0) {
      tl_lane->ctr.messages_lost++;
      on_fd_event(target, SUSPECT, k);
      continue;
    }
    Msg m;
    m.extra = (uint32_t)e;
    m.kind = K_PING_REQ;
    m.src = id;
    m.dst = h;
    m.cid_iss = id;
    m.cid_cnt = cnt;
    m.pd_from = id;
    m.pd_to = target;
    send(std::move(m), k);
    subs.push_back(Sub{cnt, 1, h, target, k + (uint64_t)timeLeft, subOrder++});
  }
}

// every pending subscription on cid `cnt` takes the first matching inbound message (TransportImpl.java:205-232)
void Member::resolve_subs(uint32_t cnt, uint64_t k) {
  std::vector<Sub> hit;
  std::vector<Sub> keep;
  for (auto& sb : subs) (sb.cnt == cnt ? hit : keep).push_back(sb);
  if (hit.empty()) return;
  subs.swap(keep);
  std::sort(hit.begin(), hit.end(), [](const Sub& a, const Sub& b) { return a.order < b.order; });
  for (auto& sb : hit) on_fd_event(sb.target, ALIVE, k);  // publishPingResult(ALIVE) (:157,202)
}

// doPing (:128-176) + selectPingMember (:338-347)
void Member::do_ping(uint64_t k) {
  Sim& s = *sim;
  fdPeriod++;
  if (ping.empty()) return;
  if (pingIdx >= (int64_t)ping.size()) {
    pingIdx = 0;
    shuffle(ping, S_FD_SHUFFLE);
  }
  uint32_t target = ping[(size_t)pingIdx++];
  uint32_t cnt = cidCnt++;
  tl_lane->ctr.messages++;
  const int e = s.xmit(K_PING, id, target, k, id, cnt, *this);
  if (e < 0) {
    tl_lane->ctr.messages_lost++;
    ping_req_step(target, cnt, k);
    return;
  }
  Msg m;
  m.extra = (uint32_t)e;
  m.kind = K_PING;
  m.src = id;
  m.dst = target;
  m.cid_iss = id;
  m.cid_cnt = cnt;
  m.pd_from = id;
  m.pd_to = target;
  send(std::move(m), k);
  subs.push_back(Sub{cnt, 0, NONE, target, k + pingTimeout_t, subOrder++});
}

// doSpreadGossip (:139-157), selectGossipMembers (:252-273), selectGossipsToSend (:239-250), sweepGossips (:283-308)
void Member::do_spread_gossip(uint64_t k) {
  Sim& s = *sim;
  uint64_t period = gPeriod++;
  if (gossips.empty()) return;
  std::vector<uint32_t> targets;
  uint32_t f = s.cfg.gossip_fanout;
  if (remote.size() < f) {
    targets = remote;
  } else {
    if (remoteIdx < 0 || remoteIdx + (int64_t)f > (int64_t)remote.size()) {
      shuffle(remote, S_GOSSIP_SHUFFLE);
      remoteIdx = 0;
    }
    targets.assign(remote.begin() + remoteIdx, remote.begin() + remoteIdx + f);
    remoteIdx += f;
  }
  uint32_t cluster = (uint32_t)remote.size() + 1;
  uint64_t sp = s.spread_of(cluster);
  for (uint32_t slot = 0; slot < targets.size(); ++slot) {
    uint32_t t = targets[slot];
    for (auto& kv : gossips) {
      GState& g = kv.second;
      if (g.infPeriod + sp < period) continue;
      if (g.is_infected(t)) continue;
      tl_lane->ctr.gossip_messages++;
      const int e = s.xmit_gossip(id, t, k, slot, kv.first, *this);
      if (s.send_log) fprintf(s.send_log, "S %llu %u %llu %u %d\n", (unsigned long long)k, id, (unsigned long long)kv.first, t, e < 0 ? 1 : 0);
      if (e < 0) continue;  // gossip losses are not counted (SEMANTICS.md §8)
      Msg m;
      m.extra = (uint32_t)e;
      m.kind = K_GOSSIP;
      m.src = id;
      m.dst = t;
      m.gid = kv.first;
      m.slot = slot;
      m.g_subj = g.subj;
      m.g_rec = g.rec;
      m.g_payload = g.payload;
      send(std::move(m), k, true);
    }
  }
  uint64_t sw = s.sweep_of(cluster);
  for (auto it = gossips.begin(); it != gossips.end();) {
    if (period > it->second.infPeriod + sw) {
      // the leave notification swept at its origin: leaveCluster's Mono completes and ClusterImpl.doShutdown
      // disposes the member and stops its transport (ClusterImpl.java:305-313, GossipProtocolImpl.java:296-306)
      if ((uint32_t)(it->first >> 32) == id && it->second.subj == id && it->second.rec.st == DEAD)
        tl_lane->leaving.push_back(id);
      if (s.send_log) fprintf(s.send_log, "W %llu %u %llu\n", (unsigned long long)k, id, (unsigned long long)it->first);
      it = gossips.erase(it);
    } else {
      ++it;
    }
  }
}

// doSync (:298-314) + selectSyncAddress (:410-421)
void Member::do_sync(uint64_t k) {
  Sim& s = *sim;
  std::vector<uint32_t> cand;
  {
    std::set<uint32_t> set(seeds.begin(), seeds.end());
    for (uint32_t subj = 0; subj < s.N; ++subj)
      if (subj != id && table[subj].st != ABSENT) set.insert(subj);
    cand.assign(set.begin(), set.end());
  }
  if (cand.empty()) return;
  uint32_t i = next_int(draw(S_SYNC_PICK), (uint32_t)cand.size());
  send_sync(K_SYNC, cand[i], NONE, 0, k);
}

// ClusterImpl.join0 (:85-152) -> MembershipProtocolImpl.start0 (:216-251), COLD_JOIN only
void Member::start(uint64_t k) {
  Sim& s = *sim;
  nextPing = k + ping_t;
  nextGossip = k + s.gossip_t;
  if (seeds.empty()) {
    nextSync = k + s.sync_t;
    return;
  }
  initActive = true;
  initDeadline = k + s.syncTimeout_t;
  uint32_t failed = 0;
  for (uint32_t sd : seeds) {
    uint32_t cnt = cidCnt++;
    initCids.insert(cnt);
    if (!send_sync(K_SYNC, sd, id, cnt, k)) failed++;
  }
  if (failed == seeds.size()) {  // Flux.mergeDelayError of all-failed requests errors -> doFinally
    initActive = false;
    nextSync = k + s.sync_t;
  }
}

static bool fd_less(const Msg& a, const Msg& b) {
  if (a.cid_iss != b.cid_iss) return a.cid_iss < b.cid_iss;
  if (a.cid_cnt != b.cid_cnt) return a.cid_cnt < b.cid_cnt;
  if (a.kind != b.kind) return a.kind < b.kind;
  return a.src < b.src;
}

void Member::process(uint64_t k, std::vector<Msg>& inbox) {
  Sim& s = *sim;
  std::vector<Rec> tickStartAll;  // SWIMREF_DEBUG: the table before P0 (what the engine's receipt filter reads)
  if (s.debug) tickStartAll = table;
  for (uint64_t p : pendingUser) spread(USER_SUBJ, Rec{}, p);  // Cluster.spreadGossip (ClusterImpl.java:208-211)
  pendingUser.clear();
  for (; pendingInc > 0; --pendingInc) {  // updateIncarnation (MembershipProtocolImpl.java:178-190), once per call
    Rec r{ALIVE, table[id].inc + 1};
    table[id] = r;
    tl_lane->ctr.row_writes++;
    spread(id, r);
  }
  if (pendingLeave) {  // leaveCluster (MembershipProtocolImpl.java:197-206): own record DEAD inc+1, spread
    pendingLeave = false;
    Rec r{DEAD, table[id].inc + 1};
    table[id] = r;
    tl_lane->ctr.row_writes++;
    spread(id, r);
  }
  std::vector<Msg*> syncm, fdm, mdm, gm;
  for (auto& m : inbox) {
    switch (m.kind) {
      case K_SYNC:
      case K_SYNC_ACK: syncm.push_back(&m); break;
      case K_PING:
      case K_PING_REQ:
      case K_PING_ACK: fdm.push_back(&m); break;
      case K_GMD_REQ:
      case K_GMD_RESP: mdm.push_back(&m); break;
      default: gm.push_back(&m);
    }
  }
  // ---- P1 SYNC / SYNC_ACK (onMessage :320-331, onSync :346-367, onSyncAck :337-343) ----
  std::sort(syncm.begin(), syncm.end(), [](Msg* a, Msg* b) { return a->src != b->src ? a->src < b->src : a->seq < b->seq; });
  std::vector<Rec> startTable;
  if (s.debug && syncm.size() > 1) {
    startTable = table;
    tickStart = &startTable;
  }
  for (Msg* m : syncm) {
    if (s.members[m->src].syncGroup != syncGroup) continue;  // checkSyncGroup (:320-321,431-437): SyncData of another group
    if (m->kind == K_SYNC) {
      int g = nextGroup++;
      groups[g] = Group{0, m->src, m->cid_iss, m->cid_cnt, 0, false, false};
      sync_membership(*m->payload, R_SYNC, g, k);
      groups[g].sealed = true;
      finish(g, false, k);
    } else if (m->cid_iss == NONE) {
      sync_membership(*m->payload, R_SYNC, -1, k);
    } else if (m->cid_iss == id && initActive && !initReceived && initCids.count(m->cid_cnt)) {
      initReceived = true;  // Flux.mergeDelayError(...).take(1) (:239-243)
      int g = nextGroup++;
      groups[g] = Group{1, NONE, NONE, 0, 0, false, false};
      sync_membership(*m->payload, R_INITIAL, g, k);
      groups[g].sealed = true;
      finish(g, false, k);
    }
  }
  tickStart = nullptr;
  // ---- P2 FD (onMessage :219-227) ----
  std::sort(fdm.begin(), fdm.end(), [](Msg* a, Msg* b) { return fd_less(*a, *b); });
  for (Msg* m : fdm) {
    if (m->kind == K_PING) {  // onPing (:230-255)
      if (m->pd_to != id) continue;
      tl_lane->ctr.messages++;
      const int e = s.xmit(K_PING_ACK, id, m->pd_from, k, m->cid_iss, m->cid_cnt, *this);
      if (e < 0) {
        tl_lane->ctr.messages_lost++;
        continue;
      }
      Msg a = *m;
      a.extra = (uint32_t)e;
      a.kind = K_PING_ACK;
      a.src = id;
      a.dst = m->pd_from;
      send(std::move(a), k);
    } else if (m->kind == K_PING_REQ) {  // onPingReq (:258-284): transit ping
      tl_lane->ctr.messages++;
      const int e = s.xmit(K_PING, id, m->pd_to, k, m->cid_iss, m->cid_cnt, *this);
      if (e < 0) {
        tl_lane->ctr.messages_lost++;
        continue;
      }
      Msg p;
      p.extra = (uint32_t)e;
      p.kind = K_PING;
      p.src = id;
      p.dst = m->pd_to;
      p.cid_iss = m->cid_iss;
      p.cid_cnt = m->cid_cnt;
      p.pd_from = id;
      p.pd_to = m->pd_to;
      p.pd_orig = m->pd_from;
      send(std::move(p), k);
    } else if (m->pd_orig != NONE) {  // onTransitPingAck (:290-315)
      tl_lane->ctr.messages++;
      const int e = s.xmit(K_PING_ACK, id, m->pd_orig, k, m->cid_iss, m->cid_cnt, *this);
      if (e < 0) {
        tl_lane->ctr.messages_lost++;
        continue;
      }
      Msg a;
      a.extra = (uint32_t)e;
      a.kind = K_PING_ACK;
      a.src = id;
      a.dst = m->pd_orig;
      a.cid_iss = m->cid_iss;
      a.cid_cnt = m->cid_cnt;
      a.pd_from = m->pd_orig;
      a.pd_to = m->pd_to;
      send(std::move(a), k);
    } else if (m->cid_iss == id) {  // response for a pending requestResponse
      resolve_subs(m->cid_cnt, k);
    }
  }
  // ---- P3 metadata (MetadataStoreImpl.onMessage :192-196, onMetadataRequest :202-241) ----
  std::sort(mdm.begin(), mdm.end(), [](Msg* a, Msg* b) { return fd_less(*a, *b); });
  for (Msg* m : mdm) {
    if (m->kind == K_GMD_REQ) {
      if (m->md_subject != id) continue;
      tl_lane->ctr.messages++;
      const int e = s.xmit(K_GMD_RESP, id, m->src, k, m->cid_iss, m->cid_cnt, *this);
      if (e < 0) {
        tl_lane->ctr.messages_lost++;
        continue;
      }
      Msg r;
      r.extra = (uint32_t)e;
      r.kind = K_GMD_RESP;
      r.src = id;
      r.dst = m->src;
      r.cid_iss = m->cid_iss;
      r.cid_cnt = m->cid_cnt;
      r.md_subject = id;
      r.md_meta = s.md_version[id];
      send(std::move(r), k);
    } else if (m->cid_iss == id) {
      auto it = fetches.find(m->cid_cnt);
      if (it == fetches.end()) continue;  // late response after timeout: subscription gone
      Fetch f = it->second;
      fetches.erase(it);
      // doOnSuccess (:563-567, :576-581): updateMetadata then sink.next
      uint32_t oldm = meta[f.subj];
      meta[f.subj] = m->md_meta;
      if (f.added)
        emit_event(SWIM_EV_ADDED, f.subj, NONE, m->md_meta, k);
      else
        emit_event(SWIM_EV_UPDATED, f.subj, oldm, m->md_meta, k);
      if (f.group >= 0) groups[f.group].remaining--;
      finish(f.group, false, k);
      do_finally(f.subj, f.r1, f.reason);
    }
  }
  // ---- P4 gossip (onGossipReq :171-183) ----
  std::sort(gm.begin(), gm.end(), [](Msg* a, Msg* b) { return a->gid != b->gid ? a->gid < b->gid : a->src < b->src; });
  bool deadStamp = false;  // SWIMREF_DEBUG: a DEAD membership record among this tick's first receipts
  if (s.debug)
    for (Msg* m : gm)
      if (!gossips.count(m->gid) && m->g_subj != USER_SUBJ && m->g_rec.st == DEAD) deadStamp = true;
  for (Msg* m : gm) {
    if (s.debug && !gossips.count(m->gid) && m->g_subj != USER_SUBJ) {  // the engine's receipt_matters rule
      const Rec r0 = tickStartAll[m->g_subj], r1 = m->g_rec;
      const bool keep = r0.st == ABSENT || is_overrides(r1, r0) || deadStamp || s.leaveRequested[m->g_subj];
      if (!keep && is_overrides(r1, table[m->g_subj])) {
        s.dbg[2]++;
        fprintf(stderr, "receipt filter miss: tick %llu member %u subject %u r1 %u/%u start %u/%u live %u/%u\n",
                (unsigned long long)k, id, m->g_subj, r1.st, r1.inc, r0.st, r0.inc, table[m->g_subj].st,
                table[m->g_subj].inc);
      }
    }
    if (s.send_log) fprintf(s.send_log, "R %llu %u %u %llu %d\n", (unsigned long long)k, id, m->src, (unsigned long long)m->gid, gossips.count(m->gid) ? 0 : 1);
    if (!gossips.count(m->gid)) {
      GState g;
      g.subj = m->g_subj;
      g.rec = m->g_rec;
      g.payload = m->g_payload;
      g.infPeriod = gPeriod;
      gossips.emplace(m->gid, std::move(g));
      if (m->g_subj == USER_SUBJ) {  // sink.next -> ClusterImpl.listenGossips (:213-216); membership filters it out
        emit_event(SWIM_EV_GOSSIP, (uint32_t)(m->gid >> 32), (uint32_t)m->g_payload, (uint32_t)(m->g_payload >> 32), k,
                   (uint32_t)m->gid);
      } else {
        tl_lane->ctr.record_compares++;
        update_membership(m->g_subj, m->g_rec, R_GOSSIP, -1, k);  // onMembershipGossip (:401-408)
      }
    }
    gossips[m->gid].add_infected(m->src);
  }
  // ---- P5 timers ----
  {
    std::vector<Sub> due;
    std::vector<Sub> keep;
    for (auto& sb : subs) (sb.deadline == k ? due : keep).push_back(sb);
    subs.swap(keep);
    std::sort(due.begin(), due.end(), [](const Sub& a, const Sub& b) { return a.cnt != b.cnt ? a.cnt < b.cnt : a.order < b.order; });
    for (auto& sb : due) {
      if (sb.kind == 0)
        ping_req_step(sb.target, sb.cnt, k);  // ping timeout -> ping-req (:159-175)
      else
        on_fd_event(sb.target, SUSPECT, k);  // ping-req timeout (:204-212)
    }
  }
  {
    std::vector<uint32_t> due;
    for (auto& kv : fetches)
      if (kv.second.deadline == k) due.push_back(kv.first);
    for (uint32_t c : due) {  // .timeout(metadataTimeout) -> onErrorResume(TimeoutException) (:568,582)
      Fetch f = fetches[c];
      fetches.erase(c);
      if (f.group >= 0) groups[f.group].remaining--;
      finish(f.group, false, k);
      do_finally(f.subj, f.r1, f.reason);
    }
  }
  if (initActive && !initReceived && k == initDeadline) {  // .timeout(syncTimeout) (:241)
    initActive = false;
    nextSync = k + s.sync_t;
  }
  {
    std::vector<uint32_t> due;
    for (auto& kv : timers)
      if (kv.second == k) due.push_back(kv.first);
    for (uint32_t subj : due) {  // onSuspicionTimeout (:608-618)
      auto it = timers.find(subj);
      if (it == timers.end() || it->second != k) continue;
      timers.erase(it);
      Rec r = table[subj];
      if (r.st != ABSENT) {
        tl_lane->ctr.record_compares++;
        update_membership(subj, Rec{DEAD, r.inc}, R_TIMEOUT, -1, k);
      }
    }
  }
  // ---- P6 periodic tasks ----
  if (k == nextPing) {
    nextPing += ping_t;
    do_ping(k);
  }
  if (k == nextGossip) {
    nextGossip += s.gossip_t;
    do_spread_gossip(k);
  }
  if (k == nextSync) {
    nextSync += s.sync_t;
    do_sync(k);
  }
}

void Sim::run_tick() {
  uint64_t k = tick;
  std::vector<Msg> arrived;
  arrived.swap(inflight[k % inflight.size()]);
  std::vector<std::vector<Msg>> inbox(N);
  for (auto& m : arrived) inbox[m.dst].push_back(std::move(m));
  const int T = threads;
  if ((int)lanes.size() != T) lanes.assign(T, Lane{});
  for (auto& l : lanes) {
    std::memset(&l.ctr, 0, sizeof(l.ctr));
    l.out.clear();
    l.events.clear();
    l.leaving.clear();
  }
  tl_lane = &lanes[0];
  for (auto& m : members)  // ClusterImpl.join0 -> start0: the initial members at tick 0, joined ones at their tick
    if (m.alive && m.startTick == k) m.start(k);
  if (cfg.mode == SWIM_MODE_RUMOR && cfg.churn_per_period && k % ping_t == 0) {
    // churn of period p (SEMANTICS.md §9): event i picks a churned member v and a live origin o != v, which spreads
    // the rumor (p << 32 | v) at P0, before the user gossips queued by the host, in event order
    const uint32_t p = (uint32_t)(k / ping_t);
    std::vector<std::vector<uint64_t>> add(N);
    for (uint32_t i = 0; i < cfg.churn_per_period; ++i) {
      P4 r = philox4x32_10(p, i, 0, 0, seed_lo ^ SALT_CHURN, seed_hi);
      const uint32_t v = next_int(r.v[0], N);
      uint32_t o = next_int(r.v[1], N - 1);
      o += o >= v ? 1u : 0u;
      if (members[o].alive) add[o].push_back(((uint64_t)p << 32) | v);
    }
    for (uint32_t o = 0; o < N; ++o)
      if (!add[o].empty()) members[o].pendingUser.insert(members[o].pendingUser.begin(), add[o].begin(), add[o].end());
  }
  auto work = [&](int part) {
    tl_lane = &lanes[part];
    const uint32_t lo = (uint32_t)((uint64_t)N * part / T), hi = (uint32_t)((uint64_t)N * (part + 1) / T);
    for (uint32_t i = lo; i < hi; ++i)
      if (members[i].alive) members[i].process(k, inbox[i]);
  };
  if (T > 1)
    pool->run(work);
  else
    work(0);
  for (auto& l : lanes) {  // member order: the lanes hold contiguous member ranges
    for (auto& m : l.out) inflight[(k + lat + m.extra) % inflight.size()].push_back(std::move(m));
    events.insert(events.end(), l.events.begin(), l.events.end());
    leaving_done.insert(leaving_done.end(), l.leaving.begin(), l.leaving.end());
    ctr.record_compares += l.ctr.record_compares;
    ctr.row_writes += l.ctr.row_writes;
    ctr.messages += l.ctr.messages;
    ctr.gossip_messages += l.ctr.gossip_messages;
    ctr.events += l.ctr.events;
    ctr.messages_lost += l.ctr.messages_lost;
    ctr.gossips_created += l.ctr.gossips_created;
    ctr.sync_merges += l.ctr.sync_merges;
  }
  for (uint32_t m : leaving_done) {  // as swim_kill between this tick and the next
    members[m].alive = false;
    members[m].gossips.clear();
  }
  leaving_done.clear();
  tick++;
  ctr.tick = tick;
}

bool ms_to_ticks(uint32_t ms, uint32_t tick_ms, uint32_t* out) {
  if (ms % tick_ms) return false;
  *out = ms / tick_ms;
  return true;
}

}  // namespace

struct swim_handle {
  Sim sim;
};

extern "C" {

__attribute__((visibility("default"))) uint32_t swim_abi_version(void) { return SWIM_ABI_VERSION; }

__attribute__((visibility("default"))) void swim_default_config(swim_config* c) {
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

__attribute__((visibility("default"))) int swim_is_overrides(uint32_t r1s, uint32_t r1i, uint32_t r0s, uint32_t r0i) {
  return is_overrides(Rec{(uint8_t)r1s, r1i}, Rec{(uint8_t)r0s, r0i}) ? 1 : 0;
}
__attribute__((visibility("default"))) uint32_t swim_ceil_log2(uint32_t n) { return bitlen(n); }

__attribute__((visibility("default"))) int swim_create(const swim_config* cfg, swim_handle** out) {
  if (!cfg || !out) return SWIM_EINVAL;
  *out = nullptr;
  const swim_config& c = *cfg;
  if (c.n_members < 1 || c.tick_ms == 0 || c.latency_ticks == 0) return SWIM_EINVAL;
  if (c.ping_timeout_ms >= c.ping_interval_ms) return SWIM_EINVAL;  // ClusterConfig.java:413-415
  if (c.gossip_fanout == 0 || c.gossip_fanout > 8 || c.n_seeds > 16) return SWIM_EINVAL;
  if (c.mode > SWIM_MODE_RUMOR || (c.mode == SWIM_MODE_RUMOR && c.init_mode != SWIM_INIT_PRECONVERGED)) return SWIM_EINVAL;
  if (c.n_dormant > c.n_members || (c.n_dormant && c.init_mode != SWIM_INIT_COLD_JOIN)) return SWIM_EINVAL;
  auto* h = new swim_handle();
  h->sim.debug = getenv("SWIMREF_DEBUG") != nullptr;
  h->sim.leaveRequested.assign(c.n_members, 0);
  if (const char* th = getenv("SWIMREF_THREADS")) h->sim.threads = std::max(1, std::min(256, atoi(th)));
  if (h->sim.threads > 1) {
    h->sim.pool.reset(new Pool());
    h->sim.pool->start(h->sim.threads);
  } else if (const char* lp = getenv("SWIMREF_SEND_LOG")) {  // single-threaded only
    h->sim.send_log = fopen(lp, "w");
  }
  Sim& s = h->sim;
  s.cfg = c;
  s.N = c.n_members;
  uint32_t st;
  bool ok = ms_to_ticks(c.ping_interval_ms, c.tick_ms, &s.ping_t) && ms_to_ticks(c.ping_timeout_ms, c.tick_ms, &s.pingTimeout_t) &&
            ms_to_ticks(c.gossip_interval_ms, c.tick_ms, &s.gossip_t) && ms_to_ticks(c.sync_interval_ms, c.tick_ms, &s.sync_t) &&
            ms_to_ticks(c.sync_timeout_ms, c.tick_ms, &s.syncTimeout_t) && ms_to_ticks(c.metadata_timeout_ms, c.tick_ms, &s.md_t);
  (void)st;
  if (!ok || s.ping_t == 0 || s.gossip_t == 0 || s.sync_t == 0) {
    delete h;
    return SWIM_EINVAL;
  }
  s.lat = c.latency_ticks;
  s.seed_lo = (uint32_t)c.seed;
  s.seed_hi = (uint32_t)(c.seed >> 32);
  std::memset(&s.ctr, 0, sizeof(s.ctr));
  s.inflight.assign(s.lat + 256, {});
  s.group.assign(s.N, 0);
  s.md_version.assign(s.N, 0);
  s.members.resize(s.N);
  // members are independent (every draw is keyed by the member id): worker threads take interleaved member ranges
  auto init_member = [&](uint32_t m) {
    Member& mb = s.members[m];
    mb.sim = &s;
    mb.id = m;
    mb.ping_t = s.ping_t;
    mb.pingTimeout_t = s.pingTimeout_t;
    mb.kreq = c.ping_req_members;
    mb.table.assign(s.N, Rec{});
    mb.meta.assign(s.N, NONE);
    // seeds: LinkedHashSet, minus self (MembershipProtocolImpl.java:160-166)
    for (uint32_t i = 0; i < c.n_seeds; ++i) {
      uint32_t sd = c.seeds[i];
      if (sd >= s.N || sd == m) continue;
      if (std::find(mb.seeds.begin(), mb.seeds.end(), sd) == mb.seeds.end()) mb.seeds.push_back(sd);
    }
    if (c.init_mode == SWIM_INIT_COLD_JOIN) {
      mb.dormant = m >= s.N - c.n_dormant;
      mb.alive = !mb.dormant;  // a process not started yet refuses connections, like a dead one
      mb.startTick = mb.dormant ? NEVER : 0;
    }
    mb.table[m] = Rec{ALIVE, 0};  // :133
    mb.tsize = 1;
    mb.meta[m] = 0;  // local metadata is always known
    if (c.init_mode == SWIM_INIT_PRECONVERGED) {
      for (uint32_t x = 0; x < s.N; ++x) {
        mb.table[x] = Rec{ALIVE, 0};
        mb.meta[x] = 0;
      }
      mb.tsize = s.N;
      uint32_t n = s.N - 1;
      for (int w = 0; w < 2; ++w) {
        uint32_t keys[4];
        for (int r = 0; r < 4; ++r) keys[r] = s.init_draw(m, 16 + 4 * (uint32_t)w + (uint32_t)r, 0);
        Feistel f(n ? n : 1, keys);
        std::vector<uint32_t>& L = w == 0 ? mb.ping : mb.remote;
        L.resize(n);
        for (uint32_t i = 0; i < n; ++i) {
          uint32_t j = f(i);
          L[i] = j < m ? j : j + 1;
        }
      }
      mb.pingIdx = 0;
      mb.remoteIdx = 0;
      mb.nextPing = 1 + s.init_draw(m, 1, 0) % mb.ping_t;
      mb.nextGossip = 1 + s.init_draw(m, 2, 0) % s.gossip_t;
      mb.nextSync = 1 + s.init_draw(m, 3, 0) % s.sync_t;
      if (c.mode == SWIM_MODE_RUMOR) mb.nextPing = mb.nextSync = NEVER;  // gossip layer only (SEMANTICS.md §9)
    }
  };
  if (s.pool) {
    const uint32_t T = (uint32_t)s.threads;
    s.pool->run([&](int w) {
      for (uint32_t b = (uint32_t)w * 64; b < s.N; b += 64 * T)
        for (uint32_t m = b; m < std::min(s.N, b + 64); ++m) init_member(m);
    });
  } else {
    for (uint32_t m = 0; m < s.N; ++m) init_member(m);
  }
  *out = h;
  return SWIM_OK;
}

__attribute__((visibility("default"))) int swim_destroy(swim_handle* h) {
  if (h && h->sim.send_log) fclose(h->sim.send_log);
  delete h;
  return SWIM_OK;
}

__attribute__((visibility("default"))) int swim_step(swim_handle* h, uint32_t n) {
  if (!h) return SWIM_EINVAL;
  for (uint32_t i = 0; i < n; ++i) h->sim.run_tick();
  return SWIM_OK;
}
__attribute__((visibility("default"))) int swim_run_periods(swim_handle* h, uint32_t n) {
  if (!h) return SWIM_EINVAL;
  return swim_step(h, n * h->sim.ping_t);
}
__attribute__((visibility("default"))) int swim_sync(swim_handle* h) { return h ? SWIM_OK : SWIM_EINVAL; }

__attribute__((visibility("default"))) int swim_kill(swim_handle* h, uint32_t m) {
  if (!h || m >= h->sim.N) return SWIM_EINVAL;
  h->sim.members[m].alive = false;
  h->sim.members[m].gossips.clear();  // a crashed process keeps nothing it could gossip again (SEMANTICS.md §1)
  return SWIM_OK;
}
__attribute__((visibility("default"))) int swim_update_incarnation(swim_handle* h, uint32_t m) {
  if (!h || m >= h->sim.N || !h->sim.members[m].alive) return SWIM_EINVAL;
  h->sim.members[m].pendingInc++;
  return SWIM_OK;
}
// include/swimhip_debug.h: member m's own record at incarnation inc (the engine's limit: 2^30)
__attribute__((visibility("default"))) int swim_debug_set_incarnation(swim_handle* h, uint32_t m, uint32_t inc) {
  if (!h || m >= h->sim.N) return SWIM_EINVAL;
  if (inc >= (1u << 30)) return SWIM_ECAPACITY;
  h->sim.members[m].table[m].inc = inc;
  return SWIM_OK;
}
__attribute__((visibility("default"))) int swim_update_metadata(swim_handle* h, uint32_t m) {
  if (!h || m >= h->sim.N || !h->sim.members[m].alive) return SWIM_EINVAL;
  h->sim.md_version[m]++;  // MetadataStoreImpl.updateMetadata (:111-132), effective for the next response
  h->sim.members[m].pendingInc++;
  return SWIM_OK;
}
__attribute__((visibility("default"))) int swim_leave(swim_handle* h, uint32_t m) {
  if (!h || m >= h->sim.N || !h->sim.members[m].alive) return SWIM_EINVAL;
  h->sim.members[m].pendingLeave = true;
  if (h->sim.leaveRequested.size() != h->sim.N) h->sim.leaveRequested.assign(h->sim.N, 0);
  h->sim.leaveRequested[m] = 1;
  return SWIM_OK;
}
__attribute__((visibility("default"))) int swim_spread_gossip(swim_handle* h, uint32_t m, uint64_t payload) {
  if (!h || m >= h->sim.N || !h->sim.members[m].alive) return SWIM_EINVAL;
  h->sim.members[m].pendingUser.push_back(payload);
  return SWIM_OK;
}
__attribute__((visibility("default"))) int swim_join(swim_handle* h, uint32_t m, const uint32_t* seeds, uint32_t n) {
  if (!h || m >= h->sim.N || n > 16 || (n && !seeds)) return SWIM_EINVAL;
  Member& mb = h->sim.members[m];
  if (!mb.dormant) return SWIM_EINVAL;
  mb.dormant = false;
  mb.alive = true;
  mb.startTick = h->sim.tick;
  mb.seeds.clear();  // LinkedHashSet of valid ids minus self (MembershipProtocolImpl.java:160-166)
  for (uint32_t i = 0; i < n; ++i)
    if (seeds[i] < h->sim.N && seeds[i] != m && std::find(mb.seeds.begin(), mb.seeds.end(), seeds[i]) == mb.seeds.end())
      mb.seeds.push_back(seeds[i]);
  return SWIM_OK;
}
__attribute__((visibility("default"))) int swim_set_member_config(swim_handle* h, uint32_t m, const swim_member_config* mc) {
  if (!h || !mc || m >= h->sim.N) return SWIM_EINVAL;
  Sim& s = h->sim;
  Member& mb = s.members[m];
  if (s.tick > 0 && !mb.dormant) return SWIM_EINVAL;  // a running member's ClusterConfig is fixed
  uint32_t pt, tt;
  if (mc->ping_timeout_ms >= mc->ping_interval_ms || mc->ping_req_members > 8 ||
      !ms_to_ticks(mc->ping_interval_ms, s.cfg.tick_ms, &pt) || !ms_to_ticks(mc->ping_timeout_ms, s.cfg.tick_ms, &tt) || pt == 0)
    return SWIM_EINVAL;
  mb.ping_t = pt;
  mb.pingTimeout_t = tt;
  mb.kreq = mc->ping_req_members;
  mb.syncGroup = mc->sync_group;
  if (s.cfg.init_mode == SWIM_INIT_PRECONVERGED && s.cfg.mode != SWIM_MODE_RUMOR)
    mb.nextPing = 1 + s.init_draw(m, 1, 0) % mb.ping_t;  // the schedule phase under the member's own interval
  return SWIM_OK;
}
__attribute__((visibility("default"))) int swim_set_default_loss(swim_handle* h, uint32_t pct) {
  if (!h || pct > 100) return SWIM_EINVAL;
  h->sim.loss = pct;
  return SWIM_OK;
}
__attribute__((visibility("default"))) int swim_set_partition(swim_handle* h, const uint32_t* g) {
  if (!h) return SWIM_EINVAL;
  if (!g) {
    h->sim.partitioned = false;
    return SWIM_OK;
  }
  h->sim.group.assign(g, g + h->sim.N);
  h->sim.partitioned = true;
  for (auto it = h->sim.custom.begin(); it != h->sim.custom.end();)  // block() overwrites cross-group custom settings
    it = g[it->first >> 32] != g[(uint32_t)it->first] ? h->sim.custom.erase(it) : std::next(it);
  return SWIM_OK;
}
__attribute__((visibility("default"))) int swim_unblock_all(swim_handle* h) {
  if (!h) return SWIM_EINVAL;
  h->sim.partitioned = false;
  h->sim.custom.clear();  // NetworkEmulator.unblockAll (:186-192)
  return SWIM_OK;
}
__attribute__((visibility("default"))) int swim_set_link_loss(swim_handle* h, uint32_t src, uint32_t dst, uint32_t pct) {
  if (!h || src >= h->sim.N || dst >= h->sim.N || pct > 100) return SWIM_EINVAL;
  h->sim.custom[((uint64_t)src << 32) | dst] = Sim::Link{pct, 0};  // setLinkSettings(dst, pct, 0) / block (:97-150)
  return SWIM_OK;
}
__attribute__((visibility("default"))) int swim_set_link_settings(swim_handle* h, uint32_t src, uint32_t dst, uint32_t pct,
                                                                  uint32_t delay_ms) {
  if (!h || src >= h->sim.N || dst >= h->sim.N || pct > 100 || !h->sim.add_delay(delay_ms)) return SWIM_EINVAL;
  h->sim.custom[((uint64_t)src << 32) | dst] = Sim::Link{pct, delay_ms};  // setLinkSettings (:97-111)
  return SWIM_OK;
}
__attribute__((visibility("default"))) int swim_set_default_link_settings(swim_handle* h, uint32_t pct, uint32_t delay_ms) {
  if (!h || pct > 100 || !h->sim.add_delay(delay_ms)) return SWIM_EINVAL;
  h->sim.loss = pct;  // setDefaultLinkSettings (:113-125)
  h->sim.delay = delay_ms;
  return SWIM_OK;
}
__attribute__((visibility("default"))) int swim_emulator_counters(swim_handle* h, uint64_t* out, size_t cap) {
  if (!h || !out || cap < 2ull * h->sim.N) return SWIM_EINVAL;
  for (uint32_t m = 0; m < h->sim.N; ++m) {
    out[2 * m] = h->sim.members[m].emSent;
    out[2 * m + 1] = h->sim.members[m].emLost;
  }
  return SWIM_OK;
}
__attribute__((visibility("default"))) int swim_unblock_link(swim_handle* h, uint32_t src, uint32_t dst) {
  if (!h || src >= h->sim.N || dst >= h->sim.N) return SWIM_EINVAL;
  h->sim.custom.erase(((uint64_t)src << 32) | dst);  // unblock (:158-175)
  return SWIM_OK;
}
__attribute__((visibility("default"))) int swim_current_tick(swim_handle* h, uint64_t* t) {
  if (!h || !t) return SWIM_EINVAL;
  *t = h->sim.tick;
  return SWIM_OK;
}

__attribute__((visibility("default"))) int swim_read_row(swim_handle* h, uint32_t obs, uint64_t* out, size_t cap) {
  if (!h || obs >= h->sim.N || cap < h->sim.N) return SWIM_EINVAL;
  const Member& mb = h->sim.members[obs];
  for (uint32_t s = 0; s < h->sim.N; ++s) {
    const Rec& r = mb.table[s];
    if (r.st == ABSENT) {
      out[s] = 0;
      continue;
    }
    uint64_t v = (uint64_t)r.inc | ((uint64_t)r.st << 32) | ((uint64_t)(mb.meta[s] != NONE) << 34);
    auto it = mb.timers.find(s);
    if (it != mb.timers.end()) v |= (it->second & ((1ull << 29) - 1)) << 35;
    out[s] = v;
  }
  return SWIM_OK;
}

static void state_hash_range(swim_handle* h, uint64_t* out, uint32_t lo, uint32_t hi);
__attribute__((visibility("default"))) int swim_state_hash(swim_handle* h, uint64_t* out, size_t cap) {
  if (!h || cap < 6ull * h->sim.N) return SWIM_EINVAL;
  Sim& s = h->sim;
  // read-only per member: SWIMREF_THREADS workers over member ranges (the full-size parity tests hash 10^5 rows)
  const uint32_t nth = (uint32_t)std::max(1, std::min<int>(s.threads, (int)(s.N / 64) + 1));
  std::vector<std::thread> th;
  for (uint32_t t = 0; t < nth; ++t)
    th.emplace_back([&, t] { state_hash_range(h, out, (uint32_t)((uint64_t)t * s.N / nth), (uint32_t)((uint64_t)(t + 1) * s.N / nth)); });
  for (auto& x : th) x.join();
  return SWIM_OK;
}

static void state_hash_range(swim_handle* h, uint64_t* out, uint32_t lo, uint32_t hi) {
  Sim& s = h->sim;
  std::vector<uint64_t> row(s.N);
  for (uint32_t m = lo; m < hi; ++m) {
    const Member& mb = s.members[m];
    swim_read_row(h, m, row.data(), s.N);
    uint64_t hr = 0;
    for (uint32_t x = 0; x < s.N; ++x)
      if (row[x]) hr += hpair(x, row[x]);
    uint64_t hf = mix64((uint64_t)mb.pingIdx ^ 0xF00Dull) + mb.ping.size();
    for (size_t p = 0; p < mb.ping.size(); ++p) hf += hpair(p | (1ull << 40), mb.ping[p]);
    uint64_t hg = mix64((uint64_t)mb.remoteIdx ^ 0xBEEFull) + mb.remote.size();
    for (size_t p = 0; p < mb.remote.size(); ++p) hg += hpair(p | (2ull << 40), mb.remote[p]);
    uint64_t hgs = 0;
    for (auto& kv : mb.gossips) hgs += hpair(kv.first, kv.second.infPeriod);
    uint64_t misc = hpair(hpair(hpair(mb.cidCnt, mb.syncSeq), mb.gCounter), mb.nextSync) + mix64(mb.fdPeriod * 3 + mb.gPeriod * 7);
    out[6 * m + 0] = hr;
    out[6 * m + 1] = hf;
    out[6 * m + 2] = hg;
    out[6 * m + 3] = mb.evHash;
    out[6 * m + 4] = hgs;
    out[6 * m + 5] = misc;
  }
}

// include/swimhip_selftest.h: the oracle's own functions on caller inputs (the engine runs its device code)
__attribute__((visibility("default"))) int swim_selftest_eval(uint32_t op, const uint32_t* in, uint32_t* out, size_t n,
                                                              uint32_t device) {
  (void)device;
  if (op > SWIM_SELFTEST_LOSS_ROLL || (n && (!in || !out))) return SWIM_EINVAL;
  for (size_t i = 0; i < n; ++i) {
    if (op == SWIM_SELFTEST_OVERRIDES) {
      const uint32_t* a = in + 4 * i;
      out[i] = is_overrides(Rec{(uint8_t)a[0], a[1]}, Rec{(uint8_t)a[2], a[3]}) ? 1u : 0u;
    } else if (op == SWIM_SELFTEST_LOSS_ROLL) {
      const uint32_t* a = in + 8 * i;
      Sim s;
      s.seed_lo = a[6];
      s.seed_hi = a[7];
      out[i] = s.loss_roll((uint8_t)a[0], a[1], a[2], a[3], a[4], a[5]);
    } else if (op == SWIM_SELFTEST_PHILOX) {
      const uint32_t* a = in + 6 * i;
      const P4 r = philox4x32_10(a[0], a[1], a[2], a[3], a[4], a[5]);
      for (int j = 0; j < 4; ++j) out[4 * i + j] = r.v[j];
    } else {
      const uint32_t* a = in + 4 * i;
      Sim s;  // the ClusterMath restatements the simulation uses (Sim::spread_of / sweep_of / suspicion_ticks)
      s.cfg.gossip_repeat_mult = a[1];
      s.cfg.suspicion_mult = a[2];
      s.ping_t = a[3];
      out[4 * i] = bitlen(a[0]);
      out[4 * i + 1] = s.spread_of(a[0]);
      out[4 * i + 2] = s.sweep_of(a[0]);
      out[4 * i + 3] = s.suspicion_ticks(a[0], a[3]);
    }
  }
  return SWIM_OK;
}

// debugging aid (not in the ABI header): SWIMREF_DEBUG counters (Sim::dbg)
__attribute__((visibility("default"))) uint64_t swimdbg_counter(swim_handle* h, uint32_t i) {
  return h && i < 4 ? h->sim.dbg[i].load() : 0;
}

// debugging aid (not in the ABI header): the scalar fields folded into the "misc" state-hash word
__attribute__((visibility("default"))) int swimdbg_scalars(swim_handle* h, uint32_t m, uint64_t* out) {
  if (!h || m >= h->sim.N) return SWIM_EINVAL;
  const Member& mb = h->sim.members[m];
  out[0] = mb.cidCnt;
  out[1] = mb.syncSeq;
  out[2] = mb.gCounter;
  out[3] = (uint64_t)mb.nextSync;
  out[4] = mb.fdPeriod;
  out[5] = mb.gPeriod;
  return SWIM_OK;
}

__attribute__((visibility("default"))) int swim_read_lists(swim_handle* h, uint32_t obs, uint32_t* fd, uint32_t* fd_len,
                                                           uint32_t* gl, uint32_t* g_len, size_t cap, int32_t* cursors) {
  if (!h || obs >= h->sim.N) return SWIM_EINVAL;
  const Member& mb = h->sim.members[obs];
  if (mb.ping.size() > cap || mb.remote.size() > cap) return SWIM_EINVAL;
  std::copy(mb.ping.begin(), mb.ping.end(), fd);
  std::copy(mb.remote.begin(), mb.remote.end(), gl);
  *fd_len = (uint32_t)mb.ping.size();
  *g_len = (uint32_t)mb.remote.size();
  cursors[0] = (int32_t)mb.pingIdx;
  cursors[1] = (int32_t)mb.remoteIdx;
  return SWIM_OK;
}

__attribute__((visibility("default"))) int swim_read_gossips(swim_handle* h, uint32_t obs, uint64_t* ids, uint32_t* inf,
                                                             size_t cap, size_t* n_out) {
  if (!h || obs >= h->sim.N || !n_out) return SWIM_EINVAL;
  const Member& mb = h->sim.members[obs];
  size_t n = 0;
  for (auto& kv : mb.gossips) {
    if (n == cap) return SWIM_ECAPACITY;
    ids[n] = kv.first;
    inf[n] = (uint32_t)kv.second.infPeriod;
    n++;
  }
  *n_out = n;
  return SWIM_OK;
}

__attribute__((visibility("default"))) int swim_drain_events(swim_handle* h, swim_event* out, size_t cap, size_t* n_out) {
  if (!h || !n_out) return SWIM_EINVAL;
  auto& ev = h->sim.events;
  std::stable_sort(ev.begin(), ev.end(), [](const swim_event& a, const swim_event& b) {
    if (a.tick != b.tick) return a.tick < b.tick;
    if (a.observer != b.observer) return a.observer < b.observer;
    return a.seq < b.seq;
  });
  size_t n = std::min(cap, ev.size());
  std::copy(ev.begin(), ev.begin() + (long)n, out);
  ev.erase(ev.begin(), ev.begin() + (long)n);
  *n_out = n;
  return SWIM_OK;
}

__attribute__((visibility("default"))) int swim_counters_get(swim_handle* h, swim_counters* out) {
  if (!h || !out) return SWIM_EINVAL;
  *out = h->sim.ctr;
  return SWIM_OK;
}

__attribute__((visibility("default"))) const char* swim_last_error(swim_handle* h) { return h ? h->sim.err.c_str() : "null handle"; }

}  // extern "C"
