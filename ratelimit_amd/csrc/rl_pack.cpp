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

namespace rlpack {

// A growable array of plain values that is never value-initialised (the
// packer writes every element it hands out) and keeps its storage across
// batches: after the first batches no call allocates.
template <typename T>
struct Buf {
  T* p = nullptr;
  size_t n = 0, cap = 0;
  ~Buf() { delete[] p; }
  void clear() { n = 0; }
  void reserve(size_t m) {
    if (m <= cap) return;
    size_t c = cap ? cap : 1024;
    while (c < m) c *= 2;
    T* q = new T[c];
    if (n) memcpy(q, p, n * sizeof(T));
    delete[] p;
    p = q;
    cap = c;
  }
  void push(T v) {
    if (n == cap) reserve(n + 1);
    p[n++] = v;
  }
  T* grow(size_t k) {  // k more elements, returned for writing
    reserve(n + k);
    T* r = p + n;
    n += k;
    return r;
  }
};

}  // namespace rlpack

using rlpack::Buf;

struct rl_packer {
  uint32_t first_rule;
  std::unordered_map<std::string, uint32_t> ids;
  std::vector<std::string> keys;
  std::string err;
  // the batch arrays (valid until the next rl_packer_pack)
  Buf<uint8_t> dom, desc, ovf, ovu;
  Buf<uint32_t> dom_off, hits, req, ent_first, desc_off, ovr, ovrule;
  Buf<int64_t> now;
  Buf<uint16_t> klen, vlen;
  std::vector<uint32_t> pend;  // descriptors of the current message whose override key waits for its domain
  std::string dkey;    // descriptorKey scratch
};

namespace {

struct Rd {
  const uint8_t* p;
  const uint8_t* e;
  bool ok = true;
  bool more() const { return ok && p < e; }
  uint64_t varint() {
    if (p < e && !(*p & 0x80)) return *p++;  // (one-byte tags and lengths: the common case)
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

// A field key of these messages: field numbers 1..3 only matter; 0 or one
// past 2^29 - 1 (the protobuf limit) makes the message malformed.
inline bool field_ok(uint64_t tag) { return (tag >> 3) != 0 && (tag >> 3) <= 0x1FFFFFFFull; }

// Small copies inline (entry keys and values are a few bytes): overlapping
// 8-byte moves instead of a libc call per field.
inline void copy_small(uint8_t* __restrict d, const uint8_t* __restrict s, size_t n) {
  if (n >= 8 && n <= 16) {
    uint64_t a, b;
    memcpy(&a, s, 8);
    memcpy(&b, s + n - 8, 8);
    memcpy(d, &a, 8);
    memcpy(d + n - 8, &b, 8);
  } else if (n > 16) {
    memcpy(d, s, n);
  } else {
    for (size_t i = 0; i < n; i++) d[i] = s[i];
  }
}

// The batch being written: raw cursors into storage reserved for the whole
// batch up front (every output array is bounded by the payload size), kept
// in registers rather than re-read through the packer after each byte store.
struct Writer {
  uint8_t* __restrict desc;
  uint16_t* __restrict klen;
  uint16_t* __restrict vlen;
  uint32_t* __restrict req;
  uint32_t* __restrict ent_first;
  uint32_t* __restrict desc_off;
  uint8_t* __restrict ovf;
  uint32_t* __restrict ovr;
  uint8_t* __restrict ovu;
  uint32_t* __restrict ovrule;
  size_t nb = 0, ne = 0, nd = 0;  // desc bytes, entries, descriptors
};

inline bool parse_entry(Rd r, Writer& w) {
  const uint8_t *key = nullptr, *val = nullptr;
  uint64_t kl = 0, vl = 0;
  while (r.more()) {
    const uint64_t tag = r.varint();
    if (!field_ok(tag)) return false;
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
  uint8_t* d = w.desc + w.nb;
  copy_small(d, key, kl);
  d[kl] = '_';
  copy_small(d + kl + 1, val, vl);
  d[kl + 1 + vl] = '_';
  w.nb += kl + vl + 2;
  w.klen[w.ne] = (uint16_t)kl;
  w.vlen[w.ne] = (uint16_t)vl;
  w.ne++;
  return true;
}

inline bool parse_descriptor(Rd r, Writer& w, uint32_t q, bool* has_limit_out) {
  bool has_limit = false;
  uint32_t rpu = 0, unit = 0;
  while (r.more()) {
    const uint64_t tag = r.varint();
    if (!field_ok(tag)) return false;
    const uint32_t f = (uint32_t)(tag >> 3), wt = tag & 7;
    if (f == 1 && wt == 2) {
      if (!parse_entry(r.sub(), w)) return false;
    } else if (f == 2 && wt == 2) {
      Rd o = r.sub();
      has_limit = true;
      while (o.more()) {
        const uint64_t t2 = o.varint();
        if (!field_ok(t2)) return false;
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
  const size_t j = w.nd++;
  w.req[j] = q;
  w.ent_first[j + 1] = (uint32_t)w.ne;
  w.desc_off[j + 1] = (uint32_t)w.nb;
  w.ovf[j] = has_limit ? 1 : 0;
  w.ovr[j] = rpu;
  w.ovu[j] = (uint8_t)(unit > 255 ? 255 : unit);
  w.ovrule[j] = 0;
  *has_limit_out = has_limit;
  return true;
}

// descriptorKey(domain, descriptor) of packed descriptor j
// (config_impl.go:300-312): domain '.' (key | key_value) joined by '.'.
void descriptor_key(rl_packer* k, const Writer& w, const uint8_t* dom, size_t dl, uint32_t j) {
  k->dkey.assign((const char*)dom, dl);
  k->dkey.push_back('.');
  const uint32_t e0 = w.ent_first[j], e1 = w.ent_first[j + 1];
  const uint8_t* p = w.desc + w.desc_off[j];
  for (uint32_t e = e0; e < e1; e++) {
    const uint32_t kl = w.klen[e], vl = w.vlen[e];
    if (e > e0) k->dkey.push_back('.');
    k->dkey.append((const char*)p, kl);
    if (vl) { k->dkey.push_back('_'); k->dkey.append((const char*)p + kl + 1, vl); }
    p += kl + vl + 2;
  }
}

uint32_t intern(rl_packer* k) {
  auto it = k->ids.find(k->dkey);
  if (it != k->ids.end()) return it->second;
  const uint32_t rule = k->first_rule + (uint32_t)k->keys.size();
  k->ids.emplace(k->dkey, rule);
  k->keys.push_back(k->dkey);
  return rule;
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
  for (uint32_t q = 0; q < n; q++)
    if (msg_off[q + 1] < msg_off[q]) {
      k->err = "packer: message offsets must be non-decreasing";
      return RL_E_INVALID;
    }
  // every output array is bounded by the payload (an entry or descriptor costs
  // it at least 2 bytes of framing and copies no more bytes than it holds):
  // one reservation per batch, then plain stores
  const uint64_t total = n ? msg_off[n] - msg_off[0] : 0;
  const size_t cap = total / 2 + 2;
  for (auto* b : {&k->dom, &k->desc}) { b->clear(); b->reserve(total + 2); }
  for (auto* b : {&k->ovf, &k->ovu}) { b->clear(); b->reserve(cap); }
  for (auto* b : {&k->req, &k->ovr, &k->ovrule, &k->ent_first, &k->desc_off}) { b->clear(); b->reserve(cap + 1); }
  k->klen.clear(); k->klen.reserve(cap);
  k->vlen.clear(); k->vlen.reserve(cap);
  k->dom_off.clear(); k->dom_off.reserve(n + 1);
  k->hits.clear(); k->hits.reserve(n + 1);
  k->now.clear(); k->now.reserve(n + 1);
  if (n) memcpy(k->now.p, now, n * sizeof(int64_t));
  Writer w{k->desc.p, k->klen.p, k->vlen.p, k->req.p, k->ent_first.p, k->desc_off.p, k->ovf.p, k->ovr.p, k->ovu.p,
           k->ovrule.p};
  w.ent_first[0] = 0;
  w.desc_off[0] = 0;
  uint8_t* __restrict domw = k->dom.p;
  uint32_t* __restrict dom_off = k->dom_off.p;
  uint32_t* __restrict hitsw = k->hits.p;
  size_t dn = 0;
  dom_off[0] = 0;
  std::vector<uint32_t>& pend = k->pend;
  for (uint32_t q = 0; q < n; q++) {
    Rd r{msgs + msg_off[q], msgs + msg_off[q + 1]};
    const uint8_t* dom = nullptr;
    size_t dl = 0;
    uint32_t hits = 0;
    pend.clear();
    // one pass over the message; override stats keys once the domain is known
    while (r.more()) {
      const uint64_t tag = r.varint();
      if (!field_ok(tag)) { r.ok = false; break; }
      const uint32_t f = (uint32_t)(tag >> 3), wt = tag & 7;
      if (f == 2 && wt == 2) {
        bool lim = false;
        if (!parse_descriptor(r.sub(), w, q, &lim)) {
          k->err = "packer: malformed descriptor in RateLimitRequest " + std::to_string(q);
          return RL_E_INVALID;
        }
        if (lim) pend.push_back((uint32_t)(w.nd - 1));  // (its stats key needs the domain)
      } else if (f == 1 && wt == 2) {
        Rd s = r.sub();
        dom = s.p;
        dl = s.e - s.p;
      } else if (f == 3 && wt == 0) {
        hits = (uint32_t)r.varint();
      } else {
        r.skip(wt);
      }
    }
    if (!r.ok) {
      k->err = "packer: malformed RateLimitRequest " + std::to_string(q);
      return RL_E_INVALID;
    }
    for (uint32_t j : pend) {
      descriptor_key(k, w, dom, dl, j);
      w.ovrule[j] = intern(k);
    }
    copy_small(domw + dn, dom, dl);
    dn += dl;
    dom_off[q + 1] = (uint32_t)dn;
    hitsw[q] = hits;
  }
  k->desc.n = w.nb;
  k->klen.n = k->vlen.n = w.ne;
  k->req.n = k->ovr.n = k->ovrule.n = k->ovf.n = k->ovu.n = w.nd;
  k->ent_first.n = k->desc_off.n = w.nd + 1;
  k->dom.n = dn;
  k->dom_off.n = n + 1;
  k->hits.n = k->now.n = n;
  memset(out, 0, sizeof *out);
  out->n_requests = n;
  out->n_descriptors = (uint32_t)w.nd;
  out->n_entries = (uint32_t)w.ne;
  out->n_rules = rl_packer_rules(k);
  out->domain_bytes = k->dom.p;
  out->domain_off = k->dom_off.p;
  out->now = k->now.p;
  out->hits = k->hits.p;
  out->req_idx = k->req.p;
  out->entry_first = k->ent_first.p;
  out->desc_off = k->desc_off.p;
  out->desc_bytes = k->desc.p;
  out->key_len = k->klen.p;
  out->value_len = k->vlen.p;
  out->override_flags = k->ovf.p;
  out->override_rpu = k->ovr.p;
  out->override_unit = k->ovu.p;
  out->override_rule = k->ovrule.p;
  k->err.clear();
  return RL_OK;
}

}  // extern "C"
