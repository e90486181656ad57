"""rf_amd_filter_print (routing_filter_print, src/routing_filter.c:1185-1286) is host-only
debug text: checked on the CPU against a Python restatement of the reference's printer,
over an oracle-built image (no GPU work)."""
import numpy as np

from splinterdb_amd import engine as E
from splinterdb_amd import keys as K


def ref_bucket_bounds(enc: bytes, length: int, bo: int):
    """routing_get_bucket_bounds (:230-279), word by word as the reference does it."""
    def word(w):
        return int.from_bytes(enc[4 * w: 4 * w + 4].ljust(4, b"\0"), "little")

    def ffs(x):
        return (x & -x).bit_length()
    if bo == 0:
        w = 0
        while word(w) == 0:
            w += 1
        return 0, 32 * w + ffs(word(w)) - 1
    w, bucket, pop = 0, 0, bin(word(0)).count("1")
    while 4 * w < length and bucket + pop < bo:
        bucket += pop
        w += 1
        pop = bin(word(w)).count("1")
    ew = word(w)
    while bucket < bo - 1:
        ew &= ew - 1
        bucket += 1
    start = 32 * w + ffs(ew) - 1 - bo + 1
    ew &= ew - 1
    while ew == 0:
        w += 1
        ew = word(w)
    return start, 32 * w + ffs(ew) - 1 - bo


def ref_print(cfg, f) -> str:
    lis, isz = cfg.log_index_size, 1 << cfg.log_index_size
    lnb = max(f.num_fingerprints.bit_length() - 1, lis)
    rem, vs = cfg.fingerprint_size - lnb, f.value_size
    rvs = rem + vs
    pg = f.pages.tobytes()
    out = ["*" * 80 + "\n", "***   filter INDEX\n", "***   filter_addr: 0\n", "-" * 80 + "\n"]
    for i in range(f.num_indices):
        out.append(f"index 0x{i:x}: {int(f.slots[i])}\n")
    for i in range(f.num_indices):
        h = int(f.slots[i])
        c = pg[h] | (pg[h + 1] << 8)
        out += ["-" * 40 + "\n", f"--- Index 0x{i:x}\n", f"--- Encoding: {c}\n"]
        enc = pg[h + 2:]
        bits = ""
        for k in range(c + isz):
            if k and k % 16 == 0:
                bits += " | "
            bits += "1" if enc[k // 8] & (1 << (k % 8)) else "0"
        out.append(bits + "\n")
        out.append("--- Remainders\n")
        hl = (c + isz - 1) // 8 + 1 + 2   # print_remainders' header_length (:1234-1236)
        data = int.from_bytes(pg[h + hl: h + hl + 8192], "little")
        for bo in range(isz):
            s, e = ref_bucket_bounds(enc, hl, bo)
            line = f"0x{bo:x} remainders:"
            for j in range(s, e):
                rv = (data >> (j * rvs)) & ((1 << rvs) - 1)  # PackedArray_get, LSB first
                line += f" 0x{rv >> vs:x}:{rv & ((1 << vs) - 1)}"
            out.append(line + "\n")
    return "".join(out)


def test_print_matches_reference_format(oracle, tmp_path):
    for n, v, lis in ((3000, 0, 8), (1500, 5, 6)):
        cfg = E.routing_config_init(log_index_size=lis)
        of = oracle.filter_add(oracle.make_config(log_index_size=lis),
                               oracle.hash_fixed(K.seq_keys(0, n).reshape(-1), 24), value=v)
        f = E.RoutingFilter(of.num_fingerprints, of.num_unique, of.value_size, of.num_indices,
                            of.num_pages, of.pages(), of.slots()[: of.num_indices].copy())
        got = E.routing_filter_print(cfg, f, str(tmp_path / "p.txt"))
        assert got == ref_print(cfg, f)
        assert got.count("remainders:") == f.num_indices * (1 << lis)
