// java/src/main/java/io/scalecube/cluster/sim/SimulatedCluster.java — the reference's public surface over one
// libswimhip handle: every simulated member is a MembershipProtocol (MembershipProtocol.java:14-65) whose listen()
// flux carries its MembershipEvents (MembershipEvent.java:39-71), and listenGossips() carries user gossips
// (Cluster.listenGossips, ClusterImpl.java:213-216). ClusterConfig is unchanged (ClusterConfig.java:24). All state
// lives on the GPU; the JVM holds one handle driven from one scheduler thread, as each reference member is confined
// to its own single-thread scheduler (ClusterImpl.java:93).
package io.scalecube.cluster.sim;

import io.scalecube.cluster.ClusterConfig;
import io.scalecube.cluster.Member;
import io.scalecube.cluster.membership.MembershipEvent;
import io.scalecube.cluster.membership.MembershipProtocol;
import io.scalecube.transport.Address;
import java.util.ArrayList;
import java.util.Collection;
import java.util.Collections;
import java.util.List;
import java.util.Map;
import java.util.Optional;
import java.util.concurrent.ConcurrentHashMap;
import reactor.core.publisher.DirectProcessor;
import reactor.core.publisher.Flux;
import reactor.core.publisher.Mono;
import reactor.core.scheduler.Scheduler;
import reactor.core.scheduler.Schedulers;

public final class SimulatedCluster implements AutoCloseable {
  private final SwimHip hip;
  private final Scheduler scheduler = Schedulers.newSingle("swimhip");
  private final Map<Integer, DirectProcessor<MembershipEvent>> membership = new ConcurrentHashMap<>();
  private final Map<Integer, DirectProcessor<long[]>> gossips = new ConcurrentHashMap<>();

  /** N members joined like {@code Cluster.join(config)}; PRECONVERGED unless {@code coldJoin}. */
  public SimulatedCluster(int members, ClusterConfig config, long seed, int gpus, boolean coldJoin) {
    this.hip = new SwimHip(members, config, seed, gpus, coldJoin);
  }

  /** The simulated member of index i: id "i", address 10.a.b.c:4801 (the identities of include/swimhip_wire.h). */
  public static Member memberOf(int i) {
    return new Member(String.valueOf(i),
        Address.create("10." + ((i >> 16) & 255) + "." + ((i >> 8) & 255) + "." + (i & 255), 4801));
  }

  static int indexOf(String id) {
    return Integer.parseInt(id);
  }

  static Map<String, String> metadata(int version) {  // metadata is modelled as a version (DESIGN.md §4)
    return version == SwimHip.META_NONE
        ? Collections.emptyMap()
        : Collections.singletonMap("version", Integer.toUnsignedString(version));
  }

  /** Advances virtual time by whole ticks on the handle's thread and publishes what every member emitted. */
  public Mono<Void> advance(int ticks) {
    return Mono.<Void>fromRunnable(
            () -> {
              hip.step(ticks);
              for (SwimHip.Event e : hip.drainEvents()) route(e);
            })
        .subscribeOn(scheduler);
  }

  private void route(SwimHip.Event e) {
    if (e.type() == SwimHip.EV_GOSSIP) {
      DirectProcessor<long[]> p = gossips.get(e.observer());
      if (p != null) {
        long payload = (Integer.toUnsignedLong(e.newMeta()) << 32) | Integer.toUnsignedLong(e.oldMeta());
        p.onNext(new long[] {e.subject(), payload});
      }
      return;
    }
    DirectProcessor<MembershipEvent> p = membership.get(e.observer());
    if (p == null) return;
    Member m = memberOf(e.subject());
    switch (e.type()) {
      case SwimHip.EV_ADDED:
        p.onNext(MembershipEvent.createAdded(m, metadata(e.newMeta())));
        break;
      case SwimHip.EV_REMOVED:
        p.onNext(MembershipEvent.createRemoved(m, metadata(e.oldMeta())));
        break;
      default:
        p.onNext(MembershipEvent.createUpdated(m, metadata(e.oldMeta()), metadata(e.newMeta())));
    }
  }

  /** Member i's MembershipProtocol. */
  public MembershipProtocol membership(int i) {
    return new Protocol(i);
  }

  /** Cluster.listenGossips() of member i: (origin index, 64-bit payload) per first receipt. */
  public Flux<long[]> listenGossips(int i) {
    return gossips.computeIfAbsent(i, k -> DirectProcessor.create());
  }

  /** Cluster.spreadGossip from member i (a 64-bit payload). */
  public void spreadGossip(int i, long payload) {
    hip.spreadGossip(i, payload);
  }

  /** Cluster.updateMetadata of member i. */
  public void updateMetadata(int i) {
    hip.updateMetadata(i);
  }

  /** The fault model of NetworkEmulator (transport/.../NetworkEmulator.java:113-192). */
  public SwimHip network() {
    return hip;
  }

  private final class Protocol implements MembershipProtocol {
    private final int self;

    Protocol(int self) {
      this.self = self;
    }

    @Override
    public Mono<Void> start() {
      return Mono.empty();  // the member runs from the handle's creation (or its swim_join)
    }

    @Override
    public void stop() {
      hip.leave(self);  // leaveCluster, then the member stops when its leave gossip is swept
    }

    @Override
    public Flux<MembershipEvent> listen() {
      return membership.computeIfAbsent(self, k -> DirectProcessor.create());
    }

    @Override
    public Collection<Member> members() {
      long[] row = hip.readRow(self);
      List<Member> out = new ArrayList<>();
      for (int s = 0; s < row.length; s++) if (row[s] != 0) out.add(memberOf(s));
      return out;
    }

    @Override
    public Collection<Member> otherMembers() {
      Collection<Member> all = members();
      all.remove(member());
      return all;
    }

    @Override
    public Member member() {
      return memberOf(self);
    }

    @Override
    public Optional<Member> member(String id) {
      int s = indexOf(id);
      return s >= 0 && s < hip.members && hip.readRow(self)[s] != 0 ? Optional.of(memberOf(s)) : Optional.empty();
    }

    @Override
    public Optional<Member> member(Address address) {
      String[] b = address.host().split("\\.");
      if (b.length != 4 || address.port() != 4801) return Optional.empty();
      int s = (Integer.parseInt(b[1]) << 16) | (Integer.parseInt(b[2]) << 8) | Integer.parseInt(b[3]);
      return member(String.valueOf(s));
    }
  }

  @Override
  public void close() {
    membership.values().forEach(p -> p.onComplete());
    gossips.values().forEach(p -> p.onComplete());
    scheduler.dispose();
    hip.close();
  }
}
