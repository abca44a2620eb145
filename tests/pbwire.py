"""Minimal protobuf wire encoder for envoy.service.ratelimit.v3.RateLimitRequest
(test infrastructure: builds the gRPC payloads the host packer parses).

  RateLimitRequest     1: domain  2: descriptors (repeated)  3: hits_addend
  RateLimitDescriptor  1: entries (repeated Entry{1: key, 2: value})  2: limit {1: requests_per_unit, 2: unit}
"""


def varint(v: int) -> bytes:
    out = bytearray()
    while True:
        b = v & 0x7F
        v >>= 7
        if v:
            out.append(b | 0x80)
        else:
            out.append(b)
            return bytes(out)


def field_bytes(f: int, data: bytes) -> bytes:
    return varint(f << 3 | 2) + varint(len(data)) + data


def field_varint(f: int, v: int) -> bytes:
    return varint(f << 3) + varint(v)


def encode_request(req, extra_unknown=False) -> bytes:
    """``req``: domain, descriptors (entries [(k, v)], limit or None), hits_addend.
    proto3 omits default values (empty strings, zero integers)."""
    out = bytearray()
    if extra_unknown:
        out += field_varint(9, 12345) + field_bytes(10, b"ignored")
    if req.domain:
        out += field_bytes(1, req.domain.encode())
    for d in req.descriptors:
        body = bytearray()
        for k, v in d.entries:
            e = (field_bytes(1, k.encode()) if k else b"") + (field_bytes(2, v.encode()) if v else b"")
            body += field_bytes(1, e)
        lim = getattr(d, "limit", None)
        if lim is not None:
            o = (field_varint(1, lim.requests_per_unit) if lim.requests_per_unit else b"") + \
                (field_varint(2, lim.unit) if lim.unit else b"")
            body += field_bytes(2, o)
        out += field_bytes(2, bytes(body))
    if req.hits_addend:
        out += field_varint(3, req.hits_addend)
    return bytes(out)
