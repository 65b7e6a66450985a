/*
 * swimhip_shard.h — row-sharded multi-GPU handles of libswimhip.
 *
 * One process per GPU. Each process creates one handle for its shard of the observers (contiguous ranges
 * [floor(r N / W), floor((r+1) N / W))). The shards advance in lockstep: every call of swim_step /
 * swim_run_periods is collective, as are swim_kill, swim_set_default_loss, swim_set_partition, swim_unblock_all
 * and swim_update_incarnation, which every rank must issue with the same arguments at the same tick.
 * Per tick the shards run two exchanges (gossip records and SYNC / SYNC_ACK payloads; first receipts and
 * sweeps). With SWIM_TRANSPORT_RCCL they are RCCL send/recv groups over xGMI on the handle's stream; with
 * SWIM_TRANSPORT_HOST the library stages the blocks through host memory and calls the caller's exchange function
 * (tests drive it with torch.distributed gloo, a Java host could drive it with its own transport).
 *
 * The reference has no counterpart: it runs one JVM process per member, which exchange messages over TCP
 * (TransportImpl.java:342-367). The membership-visible behaviour of a sharded handle is identical to the
 * single-GPU handle of include/swimhip.h: the readback calls (swim_read_row, swim_read_lists, swim_read_gossips,
 * swim_state_hash, swim_drain_events, swim_counters_get) report this shard's observers only; swim_state_hash
 * leaves the other observers' words zero, and the counters are this shard's share (their sum over the ranks is the
 * whole simulation's).
 */
#ifndef SWIMHIP_SHARD_H
#define SWIMHIP_SHARD_H

#include "swimhip.h"

#ifdef __cplusplus
extern "C" {
#endif

#define SWIM_TRANSPORT_RCCL 1u
#define SWIM_TRANSPORT_HOST 2u

/* Host exchange: an all-to-all of one byte block per peer. `send` holds the blocks for ranks 0..world-1 back to
 * back; send_bytes[q] describes the block for rank q: its size in bytes in bits 0..47 and flags in bits 48..63
 * (the caller's own block is empty). The callee writes the blocks received from ranks 0..world-1 back to back
 * into `recv` (at most recv_cap bytes) and sets recv_bytes[p] to the word rank p sent for it (size and flags
 * unchanged). Returns 0 on success. Called from inside swim_step on the stepping thread. */
#define SWIM_XCOUNT_MASK ((1ull << 48) - 1)
typedef int (*swim_exchange_fn)(void* ctx, const void* send, const uint64_t* send_bytes, void* recv, uint64_t recv_cap,
                                uint64_t* recv_bytes);

typedef struct swim_shard_spec {
  uint32_t rank;
  uint32_t world;
  uint32_t transport;   /* SWIM_TRANSPORT_RCCL | SWIM_TRANSPORT_HOST */
  uint32_t chunk_cap;   /* SYNC payload chunks (2048 records each) per peer per tick; 0 = default */
  uint8_t rccl_id[128]; /* RCCL: ncclUniqueId from swim_rccl_unique_id on rank 0, broadcast by the caller */
  swim_exchange_fn exchange; /* HOST */
  void* ctx;                 /* HOST */
  uint32_t reserved[8];
} swim_shard_spec;

/* an RCCL unique id (NCCL_UNIQUE_ID_BYTES = 128) for swim_shard_spec.rccl_id; call on rank 0 only */
int swim_rccl_unique_id(uint8_t* out128);
/* collective over the `world` ranks; cfg->n_gpus is ignored, cfg->device is this rank's HIP device */
int swim_create_sharded(const swim_config* cfg, const swim_shard_spec* spec, swim_handle** out);
/* the observers this handle owns: [*lo, *hi) */
int swim_shard_range(swim_handle* h, uint32_t* lo, uint32_t* hi);

#ifdef __cplusplus
}
#endif
#endif
