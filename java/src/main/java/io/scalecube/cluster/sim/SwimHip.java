// java/src/main/java/io/scalecube/cluster/sim/SwimHip.java — the reference-side binding of libswimhip (Panama FFM,
// JDK 21+, run with --enable-native-access=ALL-UNNAMED). It binds every entry point of include/swimhip.h that the
// facade below needs; the struct layouts mirror the C structs field for field (tests/test_java_binding.py checks the
// names, order and offsets against the ctypes mirror, since this image has no JDK to compile it).
package io.scalecube.cluster.sim;

import static java.lang.foreign.ValueLayout.ADDRESS;
import static java.lang.foreign.ValueLayout.JAVA_INT;
import static java.lang.foreign.ValueLayout.JAVA_LONG;

import io.scalecube.cluster.ClusterConfig;
import java.lang.foreign.Arena;
import java.lang.foreign.FunctionDescriptor;
import java.lang.foreign.Linker;
import java.lang.foreign.MemoryLayout;
import java.lang.foreign.MemoryLayout.PathElement;
import java.lang.foreign.MemorySegment;
import java.lang.foreign.SymbolLookup;
import java.lang.invoke.MethodHandle;

/** One libswimhip handle: N simulated scalecube members, each configured like {@code Cluster.join(config)}. */
public final class SwimHip implements AutoCloseable {
  private static final Linker LINKER = Linker.nativeLinker();
  private static final SymbolLookup LIB =
      SymbolLookup.libraryLookup(System.getProperty("swimhip.lib", "libswimhip.so"), Arena.global());

  private static MethodHandle fn(String name, FunctionDescriptor d) {
    return LINKER.downcallHandle(LIB.find(name).orElseThrow(), d);
  }

  /** include/swimhip.h swim_config: 192 bytes (8-byte aligned: 4 bytes of tail padding). */
  static final MemoryLayout CONFIG =
      MemoryLayout.structLayout(
          JAVA_INT.withName("n_members"),
          JAVA_INT.withName("tick_ms"),
          JAVA_INT.withName("latency_ticks"),
          JAVA_INT.withName("init_mode"),
          JAVA_LONG.withName("seed"),
          JAVA_INT.withName("sync_interval_ms"),
          JAVA_INT.withName("sync_timeout_ms"),
          JAVA_INT.withName("suspicion_mult"),
          JAVA_INT.withName("ping_interval_ms"),
          JAVA_INT.withName("ping_timeout_ms"),
          JAVA_INT.withName("ping_req_members"),
          JAVA_INT.withName("gossip_interval_ms"),
          JAVA_INT.withName("gossip_fanout"),
          JAVA_INT.withName("gossip_repeat_mult"),
          JAVA_INT.withName("metadata_timeout_ms"),
          JAVA_INT.withName("mode"),
          JAVA_INT.withName("flags"),
          JAVA_INT.withName("n_seeds"),
          MemoryLayout.sequenceLayout(16, JAVA_INT).withName("seeds"),
          JAVA_INT.withName("gossip_slot_cap"),
          JAVA_INT.withName("pending_fetch_cap"),
          JAVA_INT.withName("event_cap"),
          JAVA_INT.withName("n_gpus"),
          JAVA_INT.withName("device"),
          JAVA_INT.withName("list_slack"),
          JAVA_INT.withName("churn_per_period"),
          JAVA_INT.withName("n_dormant"),
          JAVA_INT.withName("gossip_ring_cap"),
          JAVA_INT.withName("delay_cap_ms"),
          MemoryLayout.sequenceLayout(2, JAVA_INT).withName("reserved"),
          MemoryLayout.paddingLayout(4));

  /** swim_member_config: 32 bytes. */
  static final MemoryLayout MEMBER_CONFIG =
      MemoryLayout.structLayout(
          JAVA_INT.withName("ping_interval_ms"),
          JAVA_INT.withName("ping_timeout_ms"),
          JAVA_INT.withName("ping_req_members"),
          JAVA_INT.withName("sync_group"),
          MemoryLayout.sequenceLayout(4, JAVA_INT).withName("reserved"));

  /** swim_event: 32 bytes. */
  static final MemoryLayout EVENT =
      MemoryLayout.structLayout(
          JAVA_INT.withName("tick"),
          JAVA_INT.withName("observer"),
          JAVA_INT.withName("seq"),
          JAVA_INT.withName("type"),
          JAVA_INT.withName("subject"),
          JAVA_INT.withName("old_meta"),
          JAVA_INT.withName("new_meta"),
          JAVA_INT.withName("pad"));

  static final int EV_ADDED = 0, EV_REMOVED = 1, EV_UPDATED = 2, EV_GOSSIP = 3;
  static final int META_NONE = 0xFFFFFFFF;
  static final int FLAG_RECORD_EVENTS = 1;

  private static final MethodHandle DEFAULTS = fn("swim_default_config", FunctionDescriptor.ofVoid(ADDRESS));
  private static final MethodHandle CREATE = fn("swim_create", FunctionDescriptor.of(JAVA_INT, ADDRESS, ADDRESS));
  private static final MethodHandle DESTROY = fn("swim_destroy", FunctionDescriptor.of(JAVA_INT, ADDRESS));
  private static final MethodHandle STEP = fn("swim_step", FunctionDescriptor.of(JAVA_INT, ADDRESS, JAVA_INT));
  private static final MethodHandle KILL = fn("swim_kill", FunctionDescriptor.of(JAVA_INT, ADDRESS, JAVA_INT));
  private static final MethodHandle LEAVE = fn("swim_leave", FunctionDescriptor.of(JAVA_INT, ADDRESS, JAVA_INT));
  private static final MethodHandle JOIN =
      fn("swim_join", FunctionDescriptor.of(JAVA_INT, ADDRESS, JAVA_INT, ADDRESS, JAVA_INT));
  private static final MethodHandle LOSS =
      fn("swim_set_default_loss", FunctionDescriptor.of(JAVA_INT, ADDRESS, JAVA_INT));
  private static final MethodHandle LINK_LOSS =
      fn("swim_set_link_loss", FunctionDescriptor.of(JAVA_INT, ADDRESS, JAVA_INT, JAVA_INT, JAVA_INT));
  private static final MethodHandle UNBLOCK =
      fn("swim_unblock_link", FunctionDescriptor.of(JAVA_INT, ADDRESS, JAVA_INT, JAVA_INT));
  private static final MethodHandle DEFAULT_LINK =
      fn("swim_set_default_link_settings", FunctionDescriptor.of(JAVA_INT, ADDRESS, JAVA_INT, JAVA_INT));
  private static final MethodHandle LINK =
      fn("swim_set_link_settings", FunctionDescriptor.of(JAVA_INT, ADDRESS, JAVA_INT, JAVA_INT, JAVA_INT, JAVA_INT));
  private static final MethodHandle EMU =
      fn("swim_emulator_counters", FunctionDescriptor.of(JAVA_INT, ADDRESS, ADDRESS, JAVA_LONG));
  private static final MethodHandle UNBLOCK_ALL = fn("swim_unblock_all", FunctionDescriptor.of(JAVA_INT, ADDRESS));
  private static final MethodHandle PARTITION =
      fn("swim_set_partition", FunctionDescriptor.of(JAVA_INT, ADDRESS, ADDRESS));
  private static final MethodHandle SPREAD =
      fn("swim_spread_gossip", FunctionDescriptor.of(JAVA_INT, ADDRESS, JAVA_INT, JAVA_LONG));
  private static final MethodHandle UPDATE_METADATA =
      fn("swim_update_metadata", FunctionDescriptor.of(JAVA_INT, ADDRESS, JAVA_INT));
  private static final MethodHandle MEMBER_CFG =
      fn("swim_set_member_config", FunctionDescriptor.of(JAVA_INT, ADDRESS, JAVA_INT, ADDRESS));
  private static final MethodHandle READ_ROW =
      fn("swim_read_row", FunctionDescriptor.of(JAVA_INT, ADDRESS, JAVA_INT, ADDRESS, JAVA_LONG));
  private static final MethodHandle DRAIN =
      fn("swim_drain_events", FunctionDescriptor.of(JAVA_INT, ADDRESS, ADDRESS, JAVA_LONG, ADDRESS));
  private static final MethodHandle TICK = fn("swim_current_tick", FunctionDescriptor.of(JAVA_INT, ADDRESS, ADDRESS));
  private static final MethodHandle ERR = fn("swim_last_error", FunctionDescriptor.of(ADDRESS, ADDRESS));

  private final Arena arena = Arena.ofShared();
  private final MemorySegment handle;
  final int members;
  final int tickMs;

  /**
   * {@code members} simulated members with the reference's ClusterConfig fields (ClusterConfig.java:27-36,57);
   * {@code gpus} > 1 row-shards them over that many devices behind this one handle (swim_config.n_gpus).
   */
  public SwimHip(int members, ClusterConfig c, long seed, int gpus, boolean coldJoin) {
    this.members = members;
    this.tickMs = 100;
    MemorySegment cfg = arena.allocate(CONFIG);
    try {
      DEFAULTS.invokeExact(cfg);
      put(cfg, "n_members", members);
      cfg.set(JAVA_LONG, CONFIG.byteOffset(PathElement.groupElement("seed")), seed);
      put(cfg, "init_mode", coldJoin ? 0 : 1);
      put(cfg, "sync_interval_ms", c.getSyncInterval());
      put(cfg, "sync_timeout_ms", c.getSyncTimeout());
      put(cfg, "suspicion_mult", c.getSuspicionMult());
      put(cfg, "ping_interval_ms", c.getPingInterval());
      put(cfg, "ping_timeout_ms", c.getPingTimeout());
      put(cfg, "ping_req_members", c.getPingReqMembers());
      put(cfg, "gossip_interval_ms", (int) c.getGossipInterval());
      put(cfg, "gossip_fanout", c.getGossipFanout());
      put(cfg, "gossip_repeat_mult", c.getGossipRepeatMult());
      put(cfg, "metadata_timeout_ms", c.getMetadataTimeout());
      put(cfg, "flags", FLAG_RECORD_EVENTS);
      put(cfg, "n_gpus", gpus);
      MemorySegment out = arena.allocate(ADDRESS);
      check((int) CREATE.invokeExact(cfg, out), MemorySegment.NULL);
      handle = out.get(ADDRESS, 0);
    } catch (Throwable t) {
      arena.close();
      throw rethrow(t);
    }
  }

  private static void put(MemorySegment cfg, String field, int v) {
    cfg.set(JAVA_INT, CONFIG.byteOffset(PathElement.groupElement(field)), v);
  }

  private static RuntimeException rethrow(Throwable t) {
    return t instanceof RuntimeException ? (RuntimeException) t : new IllegalStateException(t);
  }

  private void check(int rc, MemorySegment h) throws Throwable {
    if (rc != 0) {
      MemorySegment msg = (MemorySegment) ERR.invokeExact(h);
      throw new IllegalStateException("libswimhip rc=" + rc + ": " + msg.reinterpret(4096).getString(0));
    }
  }

  private void call(int rc) {
    try {
      check(rc, handle);
    } catch (Throwable t) {
      throw rethrow(t);
    }
  }

  public void step(int ticks) {
    try {
      call((int) STEP.invokeExact(handle, ticks));
    } catch (Throwable t) {
      throw rethrow(t);
    }
  }

  public long tick() {
    try (Arena a = Arena.ofConfined()) {
      MemorySegment t = a.allocate(JAVA_LONG);
      call((int) TICK.invokeExact(handle, t));
      return t.get(JAVA_LONG, 0);
    } catch (Throwable t) {
      throw rethrow(t);
    }
  }

  /** A crashed member (no leave). */
  public void kill(int m) {
    try {
      call((int) KILL.invokeExact(handle, m));
    } catch (Throwable t) {
      throw rethrow(t);
    }
  }

  /** Cluster.shutdown(): leaveCluster, stop when the leave gossip is swept (ClusterImpl.java:297-313). */
  public void leave(int m) {
    try {
      call((int) LEAVE.invokeExact(handle, m));
    } catch (Throwable t) {
      throw rethrow(t);
    }
  }

  /** Cluster.join of a dormant member with its own seedMembers (ClusterImpl.java:85-152). */
  public void join(int m, int... seeds) {
    try (Arena a = Arena.ofConfined()) {
      MemorySegment s = a.allocate(JAVA_INT, Math.max(1, seeds.length));
      for (int i = 0; i < seeds.length; i++) s.setAtIndex(JAVA_INT, i, seeds[i]);
      call((int) JOIN.invokeExact(handle, m, s, seeds.length));
    } catch (Throwable t) {
      throw rethrow(t);
    }
  }

  /** NetworkEmulator.setDefaultLinkSettings(loss, 0) on every member. */
  public void setDefaultLoss(int pct) {
    try {
      call((int) LOSS.invokeExact(handle, pct));
    } catch (Throwable t) {
      throw rethrow(t);
    }
  }

  /** member src's NetworkEmulator.setLinkSettings(dst, loss, 0); loss 100 = block(dst). */
  public void setLinkLoss(int src, int dst, int pct) {
    try {
      call((int) LINK_LOSS.invokeExact(handle, src, dst, pct));
    } catch (Throwable t) {
      throw rethrow(t);
    }
  }

  /** NetworkEmulator.setDefaultLinkSettings(loss, meanDelay) on every member (NetworkEmulator.java:113-125). */
  public void setDefaultLinkSettings(int pct, int meanDelayMs) {
    try {
      call((int) DEFAULT_LINK.invokeExact(handle, pct, meanDelayMs));
    } catch (Throwable t) {
      throw rethrow(t);
    }
  }

  /** member src's NetworkEmulator.setLinkSettings(dst, loss, meanDelay) (NetworkEmulator.java:97-111). */
  public void setLinkSettings(int src, int dst, int pct, int meanDelayMs) {
    try {
      call((int) LINK.invokeExact(handle, src, dst, pct, meanDelayMs));
    } catch (Throwable t) {
      throw rethrow(t);
    }
  }

  /** every member's (totalMessageSentCount, totalMessageLostCount), NetworkEmulator.java:200-222. */
  public long[] emulatorCounters() {
    try (Arena a = Arena.ofConfined()) {
      MemorySegment out = a.allocate(JAVA_LONG, 2L * members);
      call((int) EMU.invokeExact(handle, out, 2L * members));
      return out.toArray(JAVA_LONG);
    } catch (Throwable t) {
      throw rethrow(t);
    }
  }

  /** member src's NetworkEmulator.unblock(dst). */
  public void unblock(int src, int dst) {
    try {
      call((int) UNBLOCK.invokeExact(handle, src, dst));
    } catch (Throwable t) {
      throw rethrow(t);
    }
  }

  /** NetworkEmulator.unblockAll() on every member. */
  public void unblockAll() {
    try {
      call((int) UNBLOCK_ALL.invokeExact(handle));
    } catch (Throwable t) {
      throw rethrow(t);
    }
  }

  /** block() of every cross-group link; null lifts the partition. */
  public void partition(int[] groupOfMember) {
    try (Arena a = Arena.ofConfined()) {
      MemorySegment g = MemorySegment.NULL;
      if (groupOfMember != null) {
        g = a.allocate(JAVA_INT, members);
        for (int i = 0; i < members; i++) g.setAtIndex(JAVA_INT, i, groupOfMember[i]);
      }
      call((int) PARTITION.invokeExact(handle, g));
    } catch (Throwable t) {
      throw rethrow(t);
    }
  }

  /** Cluster.spreadGossip(message) from member m; receipts come back as EV_GOSSIP records. */
  public void spreadGossip(int m, long payload) {
    try {
      call((int) SPREAD.invokeExact(handle, m, payload));
    } catch (Throwable t) {
      throw rethrow(t);
    }
  }

  /** Cluster.updateMetadata of member m: a new metadata version and an incarnation bump. */
  public void updateMetadata(int m) {
    try {
      call((int) UPDATE_METADATA.invokeExact(handle, m));
    } catch (Throwable t) {
      throw rethrow(t);
    }
  }

  /** Member m's own ClusterConfig: FD timings and syncGroup id (before the first step, or before its join). */
  public void setMemberConfig(int m, ClusterConfig c, int syncGroupId) {
    try (Arena a = Arena.ofConfined()) {
      MemorySegment mc = a.allocate(MEMBER_CONFIG);
      mc.set(JAVA_INT, 0, c.getPingInterval());
      mc.set(JAVA_INT, 4, c.getPingTimeout());
      mc.set(JAVA_INT, 8, c.getPingReqMembers());
      mc.set(JAVA_INT, 12, syncGroupId);
      call((int) MEMBER_CFG.invokeExact(handle, m, mc));
    } catch (Throwable t) {
      throw rethrow(t);
    }
  }

  /** observer's membership table: keys[s] = inc | status << 32 | metadata << 34 | deadline << 35, 0 = absent. */
  public long[] readRow(int observer) {
    try (Arena a = Arena.ofConfined()) {
      MemorySegment row = a.allocate(JAVA_LONG, members);
      call((int) READ_ROW.invokeExact(handle, observer, row, (long) members));
      return row.toArray(JAVA_LONG);
    } catch (Throwable t) {
      throw rethrow(t);
    }
  }

  /** One drained event record: the fields of swim_event. */
  public record Event(int tick, int observer, int seq, int type, int subject, int oldMeta, int newMeta) {}

  /** Every event emitted since the last drain, in (tick, observer, seq) order. */
  public java.util.List<Event> drainEvents() {
    java.util.List<Event> out = new java.util.ArrayList<>();
    final long cap = 65536;
    try (Arena a = Arena.ofConfined()) {
      MemorySegment buf = a.allocate(EVENT, cap);
      MemorySegment n = a.allocate(JAVA_LONG);
      long got;
      do {
        call((int) DRAIN.invokeExact(handle, buf, cap, n));
        got = n.get(JAVA_LONG, 0);
        for (long i = 0; i < got; i++) {
          MemorySegment e = buf.asSlice(i * EVENT.byteSize(), EVENT.byteSize());
          out.add(new Event(e.get(JAVA_INT, 0), e.get(JAVA_INT, 4), e.get(JAVA_INT, 8), e.get(JAVA_INT, 12),
              e.get(JAVA_INT, 16), e.get(JAVA_INT, 20), e.get(JAVA_INT, 24)));
        }
      } while (got == cap);
    } catch (Throwable t) {
      throw rethrow(t);
    }
    return out;
  }

  @Override
  public void close() {
    try {
      call((int) DESTROY.invokeExact(handle));
    } catch (Throwable t) {
      throw rethrow(t);
    } finally {
      arena.close();
    }
  }
}
