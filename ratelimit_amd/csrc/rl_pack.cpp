// rl_pack.cpp — host packer: serialized
// envoy.service.ratelimit.v3.RateLimitRequest messages, as the gRPC server
// receives them, parsed straight into the rl_request_batch arrays of
// rl_do_limit_requests, so the host never builds per-descriptor objects.
//
// Wire format (proto3; go-control-plane v0.9.7 rls.proto / ratelimit.proto):
//   RateLimitRequest      1: domain (string)  2: descriptors (repeated message)  3: hits_addend (uint32)
//   RateLimitDescriptor   1: entries (repeated message)  2: limit (RateLimitOverride)
//   Entry                 1: key (string)  2: value (string)
//   RateLimitOverride     1: requests_per_unit (uint32)  2: unit (enum)
// Unknown fields are skipped by wire type; a truncated or malformed message
// fails the call with RL_E_INVALID. An override's stats key is
// descriptorKey(domain, descriptor) (src/config/config_impl.go:300-312),
// interned here to a dense rule id; rl_packer_rule_key names it for the caller's
// stats sink.
#include <stdint.h>
#include <string.h>

#include <string>
#include <unordered_map>
#include <vector>

#include "../../include/ratelimit_hip.h"

struct rl_packer {
  uint32_t first_rule;
  std::unordered_map<std::string, uint32_t> ids;
  std::vector<std::string> keys;
  std::string err;
  // the batch arrays (valid until the next rl_packer_pack)
  std::vector<uint8_t> dom, desc, ovf, ovu;
  std::vector<uint32_t> dom_off, hits, req, ent_first, desc_off, ovr, ovrule;
  std::vector<int64_t> now;
  std::vector<uint16_t> klen, vlen;
  std::string dkey;  // descriptorKey scratch
};

namespace {

struct Rd {
  const uint8_t* p;
  const uint8_t* e;
  bool ok = true;
  bool more() const { return ok && p < e; }
  uint64_t varint() {
    uint64_t v = 0;
    for (int s = 0; s < 64; s += 7) {
      if (p >= e) { ok = false; return 0; }
      const uint8_t b = *p++;
      v |= (uint64_t)(b & 0x7F) << s;
      if (!(b & 0x80)) return v;
    }
    ok = false;
    return 0;
  }
  // a length-delimited field's bytes
  Rd sub() {
    const uint64_t n = varint();
    if (!ok || n > (uint64_t)(e - p)) { ok = false; return Rd{p, p}; }
    Rd r{p, p + n};
    p += n;
    return r;
  }
  void skip(uint32_t wt) {
    if (wt == 0) varint();
    else if (wt == 1) { if (e - p < 8) ok = false; else p += 8; }
    else if (wt == 2) sub();
    else if (wt == 5) { if (e - p < 4) ok = false; else p += 4; }
    else ok = false;  // groups (3, 4) are not used by these messages
  }
};

bool parse_entry(Rd r, rl_packer* k) {
  const uint8_t *key = nullptr, *val = nullptr;
  uint64_t kl = 0, vl = 0;
  while (r.more()) {
    const uint64_t tag = r.varint();
    const uint32_t f = (uint32_t)(tag >> 3), wt = tag & 7;
    if ((f == 1 || f == 2) && wt == 2) {
      Rd s = r.sub();
      if (f == 1) { key = s.p; kl = s.e - s.p; }
      else { val = s.p; vl = s.e - s.p; }
    } else {
      r.skip(wt);
    }
  }
  if (!r.ok || kl > 0xFFFF || vl > 0xFFFF) return false;
  const size_t o = k->desc.size();
  k->desc.resize(o + kl + vl + 2);
  uint8_t* d = k->desc.data() + o;
  if (kl) memcpy(d, key, kl);
  d[kl] = '_';
  if (vl) memcpy(d + kl + 1, val, vl);
  d[kl + 1 + vl] = '_';
  k->klen.push_back((uint16_t)kl);
  k->vlen.push_back((uint16_t)vl);
  return true;
}

// descriptorKey(domain, descriptor) from the entries just packed
// (config_impl.go:300-312): domain '.' (key | key_value) joined by '.'.
void descriptor_key(rl_packer* k, const uint8_t* dom, size_t dl, uint32_t e0, size_t b0) {
  k->dkey.assign((const char*)dom, dl);
  k->dkey.push_back('.');
  const uint8_t* p = k->desc.data() + b0;
  for (uint32_t e = e0; e < k->klen.size(); e++) {
    const uint32_t kl = k->klen[e], vl = k->vlen[e];
    if (e > e0) k->dkey.push_back('.');
    k->dkey.append((const char*)p, kl);
    if (vl) { k->dkey.push_back('_'); k->dkey.append((const char*)p + kl + 1, vl); }
    p += kl + vl + 2;
  }
}

bool parse_descriptor(Rd r, rl_packer* k, uint32_t q, const uint8_t* dom, size_t dl) {
  bool has_limit = false;
  uint32_t rpu = 0, unit = 0;
  const uint32_t e0 = (uint32_t)k->klen.size();
  const size_t b0 = k->desc.size();
  while (r.more()) {
    const uint64_t tag = r.varint();
    const uint32_t f = (uint32_t)(tag >> 3), wt = tag & 7;
    if (f == 1 && wt == 2) {
      if (!parse_entry(r.sub(), k)) return false;
    } else if (f == 2 && wt == 2) {
      Rd o = r.sub();
      has_limit = true;
      while (o.more()) {
        const uint64_t t2 = o.varint();
        const uint32_t f2 = (uint32_t)(t2 >> 3), w2 = t2 & 7;
        if (f2 == 1 && w2 == 0) rpu = (uint32_t)o.varint();
        else if (f2 == 2 && w2 == 0) unit = (uint32_t)o.varint();
        else o.skip(w2);
      }
      if (!o.ok) return false;
    } else {
      r.skip(wt);
    }
  }
  if (!r.ok) return false;
  k->req.push_back(q);
  k->ent_first.push_back((uint32_t)k->klen.size());
  k->desc_off.push_back((uint32_t)k->desc.size());
  k->ovf.push_back(has_limit ? 1 : 0);
  k->ovr.push_back(rpu);
  k->ovu.push_back((uint8_t)(unit > 255 ? 255 : unit));
  uint32_t rule = 0;
  if (has_limit) {
    descriptor_key(k, dom, dl, e0, b0);
    auto it = k->ids.find(k->dkey);
    if (it == k->ids.end()) {
      rule = k->first_rule + (uint32_t)k->keys.size();
      k->ids.emplace(k->dkey, rule);
      k->keys.push_back(k->dkey);
    } else {
      rule = it->second;
    }
  }
  k->ovrule.push_back(rule);
  return true;
}

}  // namespace

extern "C" {

rl_packer* rl_packer_create(uint32_t first_override_rule) {
  rl_packer* k = new rl_packer();
  k->first_rule = first_override_rule;
  return k;
}

void rl_packer_destroy(rl_packer* k) { delete k; }

const char* rl_packer_last_error(const rl_packer* k) { return k ? k->err.c_str() : "null packer"; }

uint32_t rl_packer_rules(const rl_packer* k) { return k ? k->first_rule + (uint32_t)k->keys.size() : 0; }

const char* rl_packer_rule_key(const rl_packer* k, uint32_t rule_id) {
  if (!k || rule_id < k->first_rule || rule_id - k->first_rule >= k->keys.size()) return nullptr;
  return k->keys[rule_id - k->first_rule].c_str();
}

int rl_packer_pack(rl_packer* k, const uint8_t* msgs, const uint64_t* msg_off, uint32_t n, const int64_t* now,
                   rl_request_batch* out) {
  if (!k || !out || (n && (!msgs || !msg_off || !now))) {
    if (k) k->err = "packer: null argument";
    return RL_E_INVALID;
  }
  k->dom.clear(); k->desc.clear(); k->ovf.clear(); k->ovu.clear();
  k->dom_off.assign(1, 0); k->hits.clear(); k->req.clear(); k->ent_first.assign(1, 0);
  k->desc_off.assign(1, 0); k->ovr.clear(); k->ovrule.clear(); k->now.assign(now, now + n);
  k->klen.clear(); k->vlen.clear();
  const uint64_t total = n ? msg_off[n] - msg_off[0] : 0;
  k->desc.reserve(total);
  k->dom.reserve(total / 8 + 16);
  for (uint32_t q = 0; q < n; q++) {
    if (msg_off[q + 1] < msg_off[q]) {
      k->err = "packer: message offsets must be non-decreasing";
      return RL_E_INVALID;
    }
    Rd r{msgs + msg_off[q], msgs + msg_off[q + 1]};
    // domain and hits first (an override's descriptorKey needs the domain)
    const uint8_t* dom = nullptr;
    size_t dl = 0;
    uint32_t hits = 0;
    Rd scan = r;
    while (scan.more()) {
      const uint64_t tag = scan.varint();
      const uint32_t f = (uint32_t)(tag >> 3), wt = tag & 7;
      if (f == 1 && wt == 2) { Rd s = scan.sub(); dom = s.p; dl = s.e - s.p; }
      else if (f == 3 && wt == 0) hits = (uint32_t)scan.varint();
      else scan.skip(wt);
    }
    if (!scan.ok) {
      k->err = "packer: malformed RateLimitRequest " + std::to_string(q);
      return RL_E_INVALID;
    }
    while (r.more()) {
      const uint64_t tag = r.varint();
      const uint32_t f = (uint32_t)(tag >> 3), wt = tag & 7;
      if (f == 2 && wt == 2) {
        if (!parse_descriptor(r.sub(), k, q, dom, dl)) {
          k->err = "packer: malformed descriptor in RateLimitRequest " + std::to_string(q);
          return RL_E_INVALID;
        }
      } else {
        r.skip(wt);
      }
    }
    if (dl) k->dom.insert(k->dom.end(), dom, dom + dl);
    k->dom_off.push_back((uint32_t)k->dom.size());
    k->hits.push_back(hits);
  }
  if (k->dom.empty()) k->dom.push_back(0);
  if (k->desc.empty()) k->desc.push_back(0);
  const uint32_t nd = (uint32_t)k->req.size();
  memset(out, 0, sizeof *out);
  out->n_requests = n;
  out->n_descriptors = nd;
  out->n_entries = (uint32_t)k->klen.size();
  out->n_rules = rl_packer_rules(k);
  out->domain_bytes = k->dom.data();
  out->domain_off = k->dom_off.data();
  out->now = k->now.data();
  out->hits = k->hits.data();
  out->req_idx = k->req.data();
  out->entry_first = k->ent_first.data();
  out->desc_off = k->desc_off.data();
  out->desc_bytes = k->desc.data();
  out->key_len = k->klen.data();
  out->value_len = k->vlen.data();
  out->override_flags = k->ovf.data();
  out->override_rpu = k->ovr.data();
  out->override_unit = k->ovu.data();
  out->override_rule = k->ovrule.data();
  k->err.clear();
  return RL_OK;
}

}  // extern "C"
