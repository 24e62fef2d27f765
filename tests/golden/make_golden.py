#!/usr/bin/env python3
"""Generate tests/golden/*.json — known-answer vectors for the echo transform.

Run from the repo root: ``python tests/golden/make_golden.py``.

Why this exists: the reference (``/root/reference/src/lib/xsk_receive.c``) cannot be compiled in
this image (``src/lib/xsk_utils.h:3`` includes libxdp's ``<xdp/xsk.h>``, which is absent) and it
ships no tests or fixtures.  The vectors here are therefore pinned by:

1. published known answers — RFC 1071 §3 numerical example, RFC 1624 §4 example (eqn 3 vs eqn 2),
   and the classic IPv4 header-checksum example (checksum 0xB861);
2. reference-run facts recorded in SURVEY.md §8a (measured by compiling the reference path in the
   survey session): csum_replace2(&c, 8, 0) equals ``~fold16(~old + 0xF7FF)`` on the big-endian
   field for all 65 536 inputs, maps 0xF7FF -> 0x0000 and never yields 0xFFFF; the gates are
   len >= 20, bytes 12-13 == 08 00, byte 23 == 1, byte 34 == 8 — IHL, version, fragment bits, ICMP
   code and checksum validity are NOT checked, and frames with 20 <= len < 42 still get bytes up
   to 37 rewritten;
3. hand-built frames whose expected outputs are computed here by an independent restatement
   written in the network-order formulation (not the C oracle's little-endian u16 code path).

The C oracle (oracle/echo_oracle.c) and the GPU kernel are both checked against these files.
classify.json holds the XDP ingress-filter action (src/kern/inner_xdp.c:26-61) of every frame, with
and without a bound AF_XDP socket, from a separate restatement (xdp_classify below).
"""
import json
import os

HERE = os.path.dirname(os.path.abspath(__file__))


def fold(s: int) -> int:
    while s >> 16:
        s = (s & 0xFFFF) + (s >> 16)
    return s


def be_sum(b: bytes, lo: int, hi: int) -> int:
    """RFC 1071 folded sum of big-endian words over b[lo:hi], odd tail zero padded."""
    s = 0
    i = lo
    while i + 1 < hi:
        s += (b[i] << 8) | b[i + 1]
        i += 2
    if i < hi:
        s += b[i] << 8
    return fold(s)


def reply_csum(old_be: int) -> int:
    """SURVEY.md §8a closed form of csum_replace2(&icmp->checksum, 8, 0) in network order."""
    return (~fold((~old_be & 0xFFFF) + 0xF7FF)) & 0xFFFF


def transform(frame: bytes, length: int):
    """Independent restatement of process_packet (xsk_receive.c:113-157) on a byte string."""
    b = bytearray(frame)
    rec = dict(verdict=1, flags=0, ip_proto=0, icmp_type=0, icmp_code=0, ip_vihl=0, eth_proto=0,
               icmp_csum_in=0, icmp_csum_out=0, ip_sum=0, icmp_sum=0)
    if length < 20:
        return bytes(b), rec
    rec.update(eth_proto=(b[12] << 8) | b[13], ip_vihl=b[14], ip_proto=b[23], icmp_type=b[34],
               icmp_code=b[35], icmp_csum_in=(b[36] << 8) | b[37])
    rec["ip_sum"] = be_sum(b, 14, min(length, 34))
    rec["icmp_sum"] = be_sum(b, 34, length) if length > 34 else 0
    if length >= 34 and rec["ip_sum"] == 0xFFFF:
        rec["flags"] |= 1
    if length >= 42 and rec["icmp_sum"] == 0xFFFF:
        rec["flags"] |= 2
    if rec["eth_proto"] != 0x0800:
        verdict = 2
    elif b[23] != 1:
        verdict = 3
    elif b[34] != 8:
        verdict = 4
    else:
        verdict = 0
        b[0:6], b[6:12] = frame[6:12], frame[0:6]
        b[26:30], b[30:34] = frame[30:34], frame[26:30]
        b[34] = 0
        new = reply_csum(rec["icmp_csum_in"])
        b[36], b[37] = new >> 8, new & 0xFF
    rec["verdict"] = verdict
    rec["icmp_csum_out"] = (b[36] << 8) | b[37]
    return bytes(b), rec


def xdp_classify(frame: bytes, length: int, bound: bool) -> int:
    """Independent restatement of xdp_sock_prog (src/kern/inner_xdp.c:26-61): 1 DROP, 2 PASS, 4 REDIRECT."""
    if length < 14:  # OVER(eth, data_end)
        return 1
    if frame[12:14] != b"\x08\x00":
        return 2
    if length < 34:  # OVER(iph, data_end)
        return 1
    if frame[23] != 1:
        return 2
    return 4 if bound else 1


def build_frame(length, *, dst=bytes.fromhex("020000000001"), src=bytes.fromhex("020000000002"),
                ethertype=0x0800, vihl=0x45, frag=0x4000, ttl=64, proto=1, saddr=bytes([10, 0, 0, 1]),
                daddr=bytes([10, 0, 0, 2]), itype=8, code=0, ident=0x1234, seq=1, payload=None,
                bad_icmp=0, bad_ip=0, window=64):
    """A frame of `length` bytes in a buffer of max(length, window) bytes (bytes past `length` are
    stale UMEM content, as in an AF_XDP chunk)."""
    size = max(length, window)
    b = bytearray((0xA0 + i) & 0xFF for i in range(size))  # stale pattern
    b[0:6] = dst
    b[6:12] = src
    b[12:14] = ethertype.to_bytes(2, "big")
    b[14] = vihl
    b[15] = 0
    b[16:18] = max(length - 14, 0).to_bytes(2, "big")
    b[18:20] = (0xBEEF).to_bytes(2, "big")
    b[20:22] = frag.to_bytes(2, "big")
    b[22] = ttl
    b[23] = proto
    b[24:26] = b"\x00\x00"
    b[26:30] = saddr
    b[30:34] = daddr
    b[34] = itype
    b[35] = code
    b[36:38] = b"\x00\x00"
    b[38:40] = ident.to_bytes(2, "big")
    b[40:42] = seq.to_bytes(2, "big")
    if payload is None:
        payload = bytes((0x10 + i) & 0xFF for i in range(max(length - 42, 0)))
    b[42:42 + len(payload)] = payload
    ipc = (~be_sum(b, 14, 34) & 0xFFFF) ^ bad_ip
    b[24:26] = ipc.to_bytes(2, "big")
    icc = (~be_sum(b, 34, max(length, 34)) & 0xFFFF) ^ bad_icmp
    b[36:38] = icc.to_bytes(2, "big")
    return bytes(b)


def frames():
    out = []

    def add(name, length, frame):
        out.append((name, length, frame))

    add("echo_64", 64, build_frame(64))
    add("echo_1500", 1500, build_frame(1500))
    add("echo_odd_len_99", 99, build_frame(99))
    # iputils ping: 56-byte payload = 8-byte timestamp + 0x10..0x37 pattern
    add("ping_iputils_98", 98, build_frame(98, ident=0x4D2, seq=7,
                                           payload=bytes.fromhex("5f5e100000000000") + bytes(range(0x10, 0x38))))
    add("ipv6_ethertype", 98, build_frame(98, ethertype=0x86DD))
    add("vlan_8100", 98, build_frame(98, ethertype=0x8100))
    add("tcp_proto6", 98, build_frame(98, proto=6))
    add("icmp_reply_type0", 98, build_frame(98, itype=0))
    add("icmp_timestamp_type13", 98, build_frame(98, itype=13))
    add("echo_code5_accepted", 98, build_frame(98, code=5))
    add("ihl6_accepted", 98, build_frame(98, vihl=0x46))
    add("version6_accepted", 98, build_frame(98, vihl=0x65))
    add("fragment_mf_accepted", 98, build_frame(98, frag=0x2000))
    add("bad_icmp_csum_accepted", 98, build_frame(98, bad_icmp=0x1234))
    add("bad_ip_csum_accepted", 98, build_frame(98, bad_ip=0x5A5A))
    add("all_zero_icmp_F7FF", 42, build_frame(42, ident=0, seq=0, payload=b""))
    add("all_zero_icmp_1500", 1500, build_frame(1500, ident=0, seq=0, payload=bytes(1458)))
    for L in (0, 1, 13, 14, 19, 20, 21, 33, 34, 37, 38, 41, 42):
        add(f"short_len_{L}", L, build_frame(L))
    return out


def main():
    vectors = []
    for name, length, frame in frames():
        out, rec = transform(frame, length)
        vectors.append(dict(name=name, len=length, input=frame.hex(), output=out.hex(), rec=rec))
    with open(os.path.join(HERE, "frames.json"), "w") as f:
        json.dump(vectors, f, indent=1)
    classify = [dict(name=name, len=length, bound=xdp_classify(frame, length, True),
                     unbound=xdp_classify(frame, length, False)) for name, length, frame in frames()]
    with open(os.path.join(HERE, "classify.json"), "w") as f:
        json.dump(classify, f, indent=1)

    kat = {
        "rfc1071_example": {"bytes": "0001f203f4f5f6f7", "folded_sum": 0xDDF2, "checksum": 0x220D},
        "rfc1624_eqn3": {"HC": 0xDD2F, "m": 0x5555, "m_new": 0x3285, "HC_new": 0x0000, "HC_new_eqn2": 0xFFFF},
        "ipv4_header_b861": {"bytes": "450000730000400040110000c0a80001c0a800c7", "checksum": 0xB861},
        # SURVEY.md §8a reference-run facts for csum_replace2(&c, ICMP_ECHO, ICMP_ECHOREPLY)
        "csum_replace2_8_0": {
            "closed_form": "new_be = ~fold16(~old_be + 0xF7FF)",
            "zero_only_from": 0xF7FF,
            "never_outputs": 0xFFFF,
            "samples": {f"{v:04x}": reply_csum(v) for v in (0x0000, 0x0001, 0x0800, 0x7FFF, 0xF7FF, 0xF800,
                                                            0xFFFE, 0xFFFF, 0x1C46, 0xB861)},
        },
    }
    with open(os.path.join(HERE, "kat.json"), "w") as f:
        json.dump(kat, f, indent=1)
    print(f"wrote {len(vectors)} frames and {len(kat)} KAT groups")


if __name__ == "__main__":
    main()
