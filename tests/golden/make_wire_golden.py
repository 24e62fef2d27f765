#!/usr/bin/env python3
"""Golden vectors for the wire-format widening (xsk_gpu_echo_dev_opts).

The reference has no such mode (process_packet reads fixed offsets, src/lib/xsk_receive.c:120-121),
so these vectors are the spec of include/xsk_gpu.h (XSK_GPU_OPT_*) computed by a second,
independent restatement in plain Python (struct + big-endian word sums, RFC 791 / 792 / 1071,
IEEE 802.1Q / 802.1ad), not by the C oracle.  The C oracle and the GPU path are checked against it.

    python tests/golden/make_wire_golden.py   ->  tests/golden/wire.json
"""
import json
import os
import struct

OPT_STRICT, OPT_VLAN, OPT_VERIFY = 1, 2, 4
TX_REPLY, DROP_SHORT, DROP_NOT_IPV4, DROP_NOT_ICMP, DROP_NOT_ECHO, DROP_BAD_DESC, DROP_BAD_IP, DROP_BAD_CSUM = range(8)
F_IP_OK, F_ICMP_OK, F_VLAN, F_OPTS = 1, 2, 4, 8


def csum16(data: bytes) -> int:
    """RFC 1071 folded sum (not complemented) of big-endian words, odd tail zero-padded."""
    if len(data) % 2:
        data = data + b"\0"
    s = sum(struct.unpack(f"!{len(data) // 2}H", data))
    while s >> 16:
        s = (s & 0xFFFF) + (s >> 16)
    return s


def build(vlan=(), ethertype=0x0800, version=4, ihl=5, options=b"", tot_len=None, frag=0x4000, proto=1,
          itype=8, code=0, ident=0x1234, seq=7, payload=b"ping", pad=0, bad_ip=False, bad_icmp=False,
          src_mac=b"\x02\x00\x00\x00\x00\x01", dst_mac=b"\x02\x00\x00\x00\x00\x02",
          saddr=b"\x0a\x00\x00\x01", daddr=b"\x0a\x00\x00\x02"):
    """An Ethernet frame carrying an IPv4 ICMP message; every field controllable."""
    icmp = bytearray(struct.pack("!BBHHH", itype, code, 0, ident, seq) + payload)
    c = (~csum16(bytes(icmp))) & 0xFFFF
    if bad_icmp:
        c ^= 0x0F0F
    icmp[2:4] = struct.pack("!H", c)
    opts = options + b"\0" * (4 * ihl - 20 - len(options)) if ihl >= 5 else b""
    hlen = 20 + len(opts)
    tl = hlen + len(icmp) if tot_len is None else tot_len
    ip = bytearray(struct.pack("!BBHHHBBH4s4s", (version << 4) | (ihl & 15), 0, tl & 0xFFFF, 0x0101, frag, 64, proto, 0,
                               saddr, daddr) + opts)
    ic = (~csum16(bytes(ip[:hlen]))) & 0xFFFF
    if bad_ip:
        ic ^= 0x00FF
    ip[10:12] = struct.pack("!H", ic)
    eth = dst_mac + src_mac
    et = ethertype
    for tpid, tci in vlan:
        eth += struct.pack("!HH", tpid, tci)
    eth += struct.pack("!H", et)
    return bytes(eth + ip + icmp + b"\0" * pad)


def expect(frame: bytes, length: int, opts: int):
    """The spec of include/xsk_gpu.h for nonzero opts: (verdict, record dict, output bytes)."""
    p = bytearray(frame)
    rec = dict(verdict=0, flags=0, ip_proto=0, icmp_type=0, icmp_code=0, ip_vihl=0, eth_proto=0, icmp_csum_in=0,
               icmp_csum_out=0, ip_sum=0, icmp_sum=0)

    def done(v):
        rec["verdict"] = v
        return v, rec, bytes(p)

    be = lambda i: (p[i] << 8) | p[i + 1]  # noqa: E731
    if length < 14:
        return done(DROP_SHORT)
    l3, et, tags = 14, be(12), 0
    if opts & OPT_VLAN:
        while tags < 2 and et in (0x8100, 0x88A8):
            if length < l3 + 4:
                return done(DROP_SHORT)
            et = be(l3 + 2)
            l3 += 4
            tags += 1
    if et != 0x0800:
        return done(DROP_NOT_IPV4)
    if length < l3 + 20:
        return done(DROP_SHORT)
    hl, end = 20, length
    if opts & OPT_STRICT:
        v, i = p[l3] >> 4, p[l3] & 15
        if v != 4 or i < 5:
            return done(DROP_BAD_IP)
        hl = 4 * i
        tot = be(l3 + 2)
        if tot < hl + 8 or l3 + tot > length:
            return done(DROP_BAD_IP)
        if be(l3 + 6) & 0x3FFF:
            return done(DROP_BAD_IP)
        end = l3 + tot
    if p[l3 + 9] != 1:
        return done(DROP_NOT_ICMP)
    l4 = l3 + hl
    if length < l4 + 8:
        return done(DROP_SHORT)
    ip_sum = csum16(bytes(p[l3:l4]))
    ic_sum = csum16(bytes(p[l4:end]))
    rec.update(eth_proto=et, ip_vihl=p[l3], ip_proto=p[l3 + 9], icmp_type=p[l4], icmp_code=p[l4 + 1],
               icmp_csum_in=be(l4 + 2), ip_sum=ip_sum, icmp_sum=ic_sum)
    fl = 0
    if ip_sum == 0xFFFF:
        fl |= F_IP_OK
    if ic_sum == 0xFFFF:
        fl |= F_ICMP_OK
    if tags:
        fl |= F_VLAN
    if hl > 20:
        fl |= F_OPTS
    rec["flags"] = fl
    if p[l4] != 8 or ((opts & OPT_STRICT) and p[l4 + 1] != 0):
        v = DROP_NOT_ECHO
    elif (opts & OPT_VERIFY) and (ip_sum != 0xFFFF or ic_sum != 0xFFFF):
        v = DROP_BAD_CSUM
    else:
        v = TX_REPLY
        p[0:6], p[6:12] = frame[6:12], frame[0:6]
        p[l3 + 12:l3 + 16], p[l3 + 16:l3 + 20] = frame[l3 + 16:l3 + 20], frame[l3 + 12:l3 + 16]
        p[l4] = 0
        # RFC 1624 eqn 3 for the 16-bit word holding type|code (type 8 -> 0): HC' = ~(~HC + ~m + m')
        old_word, new_word = (8 << 8) | p[l4 + 1], (0 << 8) | p[l4 + 1]
        hc = be(l4 + 2)
        s = ((~hc) & 0xFFFF) + ((~old_word) & 0xFFFF) + new_word
        while s >> 16:
            s = (s & 0xFFFF) + (s >> 16)
        new = (~s) & 0xFFFF
        p[l4 + 2:l4 + 4] = struct.pack("!H", new)
    rec["icmp_csum_out"] = be(l4 + 2)
    return done(v)


def cases():
    big = bytes((i * 37 + 11) & 0xFF for i in range(1400))
    c = {}
    c["plain"] = build()
    c["plain_1500"] = build(payload=big[:1472])
    c["odd_payload"] = build(payload=b"abcde")
    c["vlan1"] = build(vlan=[(0x8100, 0x0064)])
    c["vlan2_qinq"] = build(vlan=[(0x88A8, 0x0005), (0x8100, 0x0064)], payload=big[:300])
    c["vlan3_too_many"] = build(vlan=[(0x8100, 1), (0x8100, 2), (0x8100, 3)])
    c["vlan_not_ip"] = build(vlan=[(0x8100, 7)], ethertype=0x86DD)
    c["ipv6"] = build(ethertype=0x86DD)
    c["ip_options"] = build(ihl=6, options=b"\x01\x01\x01\x00")
    c["ip_options_max"] = build(ihl=15, options=b"\x07\x27\x04" + b"\0" * 37, payload=big[:100])
    c["vlan2_ihl15"] = build(vlan=[(0x88A8, 9), (0x8100, 10)], ihl=15, options=b"\x01" * 40, payload=big[:64])
    c["ihl4"] = build(ihl=4)
    c["version6"] = build(version=6)
    c["fragment_mf"] = build(frag=0x2000)
    c["fragment_off"] = build(frag=0x0010)
    c["df_only"] = build(frag=0x4000)
    c["tot_len_short"] = build(tot_len=27)
    c["tot_len_long"] = build(tot_len=200)
    c["eth_padding"] = build(payload=b"", pad=18)  # 60-B minimum frame, tot_len 28
    c["not_icmp"] = build(proto=6)
    c["echo_reply_in"] = build(itype=0)
    c["code5"] = build(code=5)
    c["bad_ip_csum"] = build(bad_ip=True)
    c["bad_icmp_csum"] = build(bad_icmp=True)
    c["zero_icmp"] = build(ident=0, seq=0, payload=b"")
    c["csum_f7ff"] = None  # filled below
    # an echo whose checksum is 0xF7FF: type 8 + everything else zero -> sum 0x0800, csum 0xF7FF
    c["csum_f7ff"] = build(ident=0, seq=0, payload=b"\0" * 32)
    fr = c["plain"]
    lens = {}
    for name, f in c.items():
        lens[name] = [len(f)]
    # truncations of interesting frames
    lens["plain"] += [0, 13, 14, 33, 34, 41, 42]
    lens["vlan1"] += [15, 17, 18, 37, 45, 46]
    lens["vlan2_qinq"] += [21, 22, 41, 49, 50]
    lens["ip_options"] += [45, 46, 49, 50]
    lens["ip_options_max"] += [80, 81, 82]
    lens["eth_padding"] += [41, 42]
    assert fr
    return c, lens


def main():
    c, lens = cases()
    out = []
    for name, f in c.items():
        for L in lens[name]:
            frame = f + b"\0" * max(0, 128 - len(f))  # window bytes past the frame: zeros
            res = {}
            for opts in range(1, 8):
                v, rec, o = expect(frame, L, opts)
                res[str(opts)] = {"verdict": v, "rec": rec, "out": o[:max(L, 1)].hex()}
            out.append({"name": name, "len": L, "frame": frame.hex(), "results": res})
    path = os.path.join(os.path.dirname(os.path.abspath(__file__)), "wire.json")
    with open(path, "w") as fh:
        json.dump(out, fh, indent=0)
    print(f"{len(out)} frames x 7 option sets -> {path}")


if __name__ == "__main__":
    main()
