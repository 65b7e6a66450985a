// wire.cpp — the Jackson JSON / length-frame encoders of include/swimhip_wire.h (host code; see the header for the
// format and its reference citations).
#include <cstdio>
#include <cstring>
#include <string>

#include "../../include/swimhip.h"
#include "../../include/swimhip_wire.h"

namespace {

const char* status_name(uint32_t st) {  // MemberStatus.toString (WRITE_ENUMS_USING_TO_STRING)
  return st == SWIM_ST_ALIVE ? "ALIVE" : st == SWIM_ST_SUSPECT ? "SUSPECT" : "DEAD";
}

void put_member(std::string& o, uint32_t m) {  // Member {id, address} (Member.java:12-13), Address {host, port}
  char b[96];
  snprintf(b, sizeof b, "{\"id\":\"%u\",\"address\":{\"host\":\"10.%u.%u.%u\",\"port\":4801}}", m, (m >> 16) & 255u,
           (m >> 8) & 255u, m & 255u);
  o += b;
}

void put_address(std::string& o, uint32_t m) {
  char b[64];
  snprintf(b, sizeof b, "{\"host\":\"10.%u.%u.%u\",\"port\":4801}", (m >> 16) & 255u, (m >> 8) & 255u, m & 255u);
  o += b;
}

// MembershipRecord: fields member, status, incarnation; is-getters alive, suspect, dead
void put_record(std::string& o, const swim_wire_record& r) {
  o += "{\"member\":";
  put_member(o, r.member);
  char b[128];
  snprintf(b, sizeof b, ",\"status\":\"%s\",\"incarnation\":%d,\"alive\":%s,\"suspect\":%s,\"dead\":%s}",
           status_name(r.status), (int)r.incarnation, r.status == SWIM_ST_ALIVE ? "true" : "false",
           r.status == SWIM_ST_SUSPECT ? "true" : "false", r.status == 3u ? "true" : "false");
  o += b;
}

void put_string(std::string& o, const char* s) {  // JSON string with the escapes Jackson writes
  o += '"';
  for (const char* p = s; *p; ++p) {
    const unsigned char c = (unsigned char)*p;
    if (c == '"' || c == '\\') {
      o += '\\';
      o += (char)c;
    } else if (c < 0x20) {
      char b[8];
      snprintf(b, sizeof b, "\\u%04X", c);
      o += b;
    } else {
      o += (char)c;
    }
  }
  o += '"';
}

int frame(const std::string& json, uint8_t* buf, size_t cap, size_t* len) {
  const size_t n = json.size();
  if (len) *len = n + 4;
  if (n > 0x7FFFFFFFu) return SWIM_ECAPACITY;
  if (!buf || cap < n + 4) return SWIM_ECAPACITY;
  buf[0] = (uint8_t)(n >> 24);  // LengthFieldPrepender: big-endian length of the payload
  buf[1] = (uint8_t)(n >> 16);
  buf[2] = (uint8_t)(n >> 8);
  buf[3] = (uint8_t)n;
  std::memcpy(buf + 4, json.data(), n);
  return SWIM_OK;
}

}  // namespace

extern "C" int swim_wire_sync_frame(uint32_t kind, uint32_t sender, const char* cid, const char* sync_group,
                                    const swim_wire_record* recs, size_t n, uint8_t* buf, size_t cap, size_t* len) {
  if ((kind != SWIM_WIRE_SYNC && kind != SWIM_WIRE_SYNC_ACK) || (n && !recs) || !len) return SWIM_EINVAL;
  std::string o;
  o.reserve(64 + n * 150);
  o += "{\"headers\":{\"q\":";  // HashMap order: "q" (hash 113) before "cid" (hash 98494)
  put_string(o, kind == SWIM_WIRE_SYNC ? "sc/membership/sync" : "sc/membership/syncAck");
  if (cid) {
    o += ",\"cid\":";
    put_string(o, cid);
  }
  o += "},\"data\":{\"@class\":\"io.scalecube.cluster.membership.SyncData\",\"membership\":[";
  for (size_t i = 0; i < n; ++i) {
    if (i) o += ',';
    put_record(o, recs[i]);
  }
  o += "],\"syncGroup\":";
  put_string(o, sync_group ? sync_group : "default");
  o += "},\"sender\":";
  put_address(o, sender);
  o += '}';
  return frame(o, buf, cap, len);
}

extern "C" int swim_wire_gossip_frame(uint32_t sender, uint32_t origin, uint32_t counter, const swim_wire_record* rec,
                                      uint8_t* buf, size_t cap, size_t* len) {
  if (!rec || !len) return SWIM_EINVAL;
  std::string o;
  char gid[32];
  snprintf(gid, sizeof gid, "%u-%u", origin, counter);
  o += "{\"headers\":{\"q\":\"sc/gossip/req\"},\"data\":{\"@class\":\"io.scalecube.cluster.gossip.GossipRequest\","
       "\"gossips\":[{\"gossipId\":";
  put_string(o, gid);
  o += ",\"message\":{\"headers\":{\"q\":\"sc/membership/gossip\"},\"data\":"
       "{\"@class\":\"io.scalecube.cluster.membership.MembershipRecord\",";
  std::string r;
  put_record(r, *rec);
  o += r.substr(1);  // the record's properties after the type id
  o += "}}],\"from\":";
  char from[16];
  snprintf(from, sizeof from, "%u", sender);
  put_string(o, from);
  o += "},\"sender\":";
  put_address(o, sender);
  o += '}';
  return frame(o, buf, cap, len);
}
