/*
 * swimhip_wire.h — wire-format export of libswimhip: the bytes the reference's TCP transport would
 * put on a connection for a simulated member's message, for trace dumps and interop.
 *
 * Frame = 4-byte big-endian length (netty LengthFieldPrepender(4), transport/.../TransportImpl.java:370-384) followed
 * by the Jackson JSON of the Message (transport/.../JacksonMessageCodec.java:41-52: every field visible, NON_NULL,
 * enums by toString, default typing JAVA_LANG_OBJECT as an "@class" property, compact output). Message fields in
 * declaration order: headers {"q", "cid"} (HashMap order of those two keys), data, sender (Message.java).
 *   SYNC / SYNC_ACK data: SyncData {membership: [MembershipRecord], syncGroup} (membership/SyncData.java:11-41,
 *     prepareSyncDataMsg MembershipProtocolImpl.java:446-454). MembershipRecord: its fields member, status,
 *     incarnation, then the is-getters alive, suspect, dead that Jackson's ANY visibility also serialises
 *     (MembershipRecord.java:12-56; their relative order follows the declaration order — HotSpot does not specify
 *     getDeclaredMethods order, so that part is parity unpinned).
 *   GOSSIP_REQ data: GossipRequest {gossips: [Gossip {gossipId, message}], from} (gossip/GossipRequest.java,
 *     Gossip.java, buildGossipRequestMessage GossipProtocolImpl.java:275-281) whose inner message is the membership
 *     gossip {headers {"q": "sc/membership/gossip"}, data: MembershipRecord} (spreadMembershipGossip :620-623).
 * Simulated identities: member i has id "<i>" (decimal) and address {"host": "10.a.b.c", "port": 4801} with a.b.c
 * the three low bytes of i (the reference's ids are random MD5 hex, IdGenerator.java:35-55, so no fixed mapping
 * exists); a gossip id is "<origin id>-<counter>" (generateGossipId, GossipProtocolImpl.java:207-209).
 * TransportConfig.DEFAULT_MAX_FRAME_LENGTH is 2 MB (TransportConfig.java:9): a SYNC of more than ~17k records
 * exceeds it, so the reference's TCP transport could not carry it; the export writes it anyway.
 */
#ifndef SWIMHIP_WIRE_H
#define SWIMHIP_WIRE_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef struct swim_handle swim_handle;

typedef struct swim_wire_record {
  uint32_t member;
  uint32_t status; /* SWIM_ST_ALIVE, SWIM_ST_SUSPECT or 3 = DEAD (a leaver's own record) */
  uint32_t incarnation;
} swim_wire_record;

#define SWIM_WIRE_SYNC 1u     /* qualifier sc/membership/sync */
#define SWIM_WIRE_SYNC_ACK 2u /* qualifier sc/membership/syncAck */

/* Encoders (host only, no handle, no device). Each writes the whole frame into buf when it fits and sets *len to the
 * frame's size either way (SWIM_ECAPACITY if cap < *len). cid: the correlation id header, or NULL for none. */
int swim_wire_sync_frame(uint32_t kind, uint32_t sender, const char* cid, const char* sync_group,
                         const swim_wire_record* records, size_t n, uint8_t* buf, size_t cap, size_t* len);
int swim_wire_gossip_frame(uint32_t sender, uint32_t origin, uint32_t counter, const swim_wire_record* record,
                           uint8_t* buf, size_t cap, size_t* len);
/* the frame of a SYNC / SYNC_ACK (cid NULL) that `observer` would send now: its live membership table, ascending by
 * member, sync group "default" */
int swim_export_sync_frame(swim_handle* h, uint32_t observer, uint32_t kind, uint8_t* buf, size_t cap, size_t* len);

#ifdef __cplusplus
}
#endif
#endif
