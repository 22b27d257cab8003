"""The GPU path against the reference's own unit tests (tests/golden/reference_cases.json,
see tests/test_reference_cases.py): every data-block case at every restart
interval it names is encoded by lsm_encode_blocks (bytes == oracle), decoded by
lsm_decode_blocks, point-read by lsm_point_read_blocks and range-sought by
lsm_seek_blocks; index-block cases round trip; hash-index bucket positions and
header checks come from the GPU's xxh3_64 / decode.  Expectations are the
reference's asserts.  One batched launch per entry point covers all cases."""
import numpy as np
import pytest

import pyoracle
from test_reference_cases import DATA, HASH, HEADER, INDEX, case_items, case_ris, check_data_case

pytestmark = pytest.mark.gpu


def _enc_gpu(gpu, items, ri, ratio, block_type=0):
    import torch
    d = gpu.items_to_device(items)
    starts = torch.tensor([0, items.n], dtype=torch.int32).cuda()
    enc = gpu.Encoder().encode(d, starts, 1, restart_interval=ri, hash_ratio=ratio, block_type=block_type)
    torch.cuda.synchronize()
    assert int(enc["status"][0]) == 0
    n = int(enc["block_off"][1])
    return enc["buf"][:n].cpu().numpy().tobytes()


def _arena(parts):
    off = np.zeros(len(parts) + 1, np.int64)
    off[1:] = np.cumsum([len(p) for p in parts])
    return b"".join(parts), off


def test_gpu_reference_data_blocks(gpu):
    import torch
    blocks, jobs = [], []  # (case, ri, payload)
    for name in sorted(DATA):
        case = DATA[name]
        items, _ = case_items(case)
        for ri in case_ris(case, cap=24):
            blk = _enc_gpu(gpu, items, ri, case["hash_ratio"])
            payload = pyoracle.data_block_encode(items, restart_interval=ri, hash_ratio=case["hash_ratio"])
            assert blk == pyoracle.block_write(payload), (name, ri)  # bit-exact vs the oracle
            jobs.append((case, ri, len(blocks), payload))
            blocks.append(blk)
    buf = b"".join(blocks)
    off = np.zeros(len(blocks) + 1, np.int64)
    off[1:] = np.cumsum([len(b) for b in blocks])
    d_buf = gpu.to_device_bytes(buf)
    d_off = torch.from_numpy(off).cuda()
    dec = gpu.decode_blocks(d_buf, d_off, len(blocks))
    torch.cuda.synchronize()
    dec = {k: v.cpu().numpy() for k, v in dec.items()}
    assert (dec["status"][:len(blocks)] == 0).all()
    # every point read / seek of every case, one launch each
    pq, sq = [], []
    for case, ri, b, payload in jobs:
        for needle, snap, _, _ in case["expect"].get("point_reads", []):
            pq.append((b, bytes.fromhex(needle), snap))
        for r in case["expect"].get("ranges", []):
            lo = None if r["lo"] is None else bytes.fromhex(r["lo"])
            hi = None if r["hi"] is None else bytes.fromhex(r["hi"])
            sq.append((b, lo, hi))
    nd, noff = _arena([q[1] for q in pq])
    pr = gpu.point_read(d_buf, d_off, len(blocks), torch.tensor([q[0] for q in pq], dtype=torch.int32).cuda(),
                        gpu.to_device_bytes(nd), torch.from_numpy(noff).cuda(),
                        torch.from_numpy(np.array([q[2] for q in pq], np.uint64).view(np.int64)).cuda())
    lo, loff = _arena([q[1] or b"" for q in sq])
    hi, hoff = _arena([q[2] or b"" for q in sq])
    flags = np.array([(1 if q[1] is not None else 0) | (2 if q[2] is not None else 0) for q in sq], np.uint8)
    sk = gpu.seek(d_buf, d_off, len(blocks), torch.tensor([q[0] for q in sq], dtype=torch.int32).cuda(),
                  gpu.to_device_bytes(lo), torch.from_numpy(loff).cuda(), gpu.to_device_bytes(hi),
                  torch.from_numpy(hoff).cuda(), torch.from_numpy(flags).cuda())
    torch.cuda.synchronize()
    pr = {k: v.cpu().numpy() for k, v in pr.items()}
    sk = {k: v.cpu().numpy() for k, v in sk.items()}
    assert (pr["status"][:len(pq)] == 0).all() and (sk["status"][:len(sq)] == 0).all()
    pi = si = 0
    for case, ri, b, payload in jobs:
        i0, i1 = int(dec["item_start"][b]), int(dec["item_start"][b + 1])
        parsed = {f: dec[f][i0:i1] for f in ("seqno", "key_off", "val_off", "val_len", "key_len", "prefix_len",
                                             "vtype")}
        parsed = {f: v.view({"seqno": np.uint64, "key_off": np.uint32, "val_off": np.uint32, "val_len": np.uint32,
                             "key_len": np.uint16, "prefix_len": np.uint16, "vtype": np.uint8}[f])
                  for f, v in parsed.items()}
        reads = {}
        for needle, snap, _, _ in case["expect"].get("point_reads", []):
            reads[(bytes.fromhex(needle), snap)] = int(pr["item"][pi])
            pi += 1
        seeks = {}
        for r in case["expect"].get("ranges", []):
            key = (r["lo"], r["hi"])
            seeks[key] = (int(sk["first"][si]), int(sk["end"][si]), bool(sk["found"][si] & 1),
                          bool(sk["found"][si] & 2))
            si += 1

        def _seek(lo_b, hi_b):
            return seeks[(None if lo_b is None else lo_b.hex(), None if hi_b is None else hi_b.hex())]

        check_data_case(case, payload, (i1 - i0, parsed), lambda nd_, sn: reads[(nd_, sn)], _seek)


def test_gpu_reference_index_blocks(gpu):
    import torch
    blocks, cases = [], []
    for name in sorted(INDEX):
        case = INDEX[name]
        keys = [bytes.fromhex(k) for k, _, _, _ in case["items"]]
        it = pyoracle.Items.from_list([(k, b"", s, 0) for k, (_, s, _, _) in zip(keys, case["items"])])
        it.handle_off = np.array([o for _, _, o, _ in case["items"]], np.uint64)
        it.handle_size = np.array([z for _, _, _, z in case["items"]], np.uint32)
        blk = _enc_gpu(gpu, it, 1, 0.0, block_type=1)
        assert blk == pyoracle.block_write(pyoracle.index_block_encode(it), 1), name
        blocks.append(blk)
        cases.append(case)
    buf = b"".join(blocks)
    off = np.zeros(len(blocks) + 1, np.int64)
    off[1:] = np.cumsum([len(b) for b in blocks])
    dec = gpu.decode_blocks(gpu.to_device_bytes(buf), torch.from_numpy(off).cuda(), len(blocks), expect_type=1)
    torch.cuda.synchronize()
    dec = {k: v.cpu().numpy() for k, v in dec.items()}
    for b, case in enumerate(cases):
        assert int(dec["status"][b]) == 0
        i0 = int(dec["item_start"][b])
        assert int(dec["item_start"][b + 1]) - i0 == case["expect"]["len"]
        pay = blocks[b][33:]
        for j, (k, s, o, z) in enumerate(case["items"]):
            ko, kl = int(dec["key_off"][i0 + j]), int(dec["key_len"][i0 + j])
            assert pay[ko:ko + kl] == bytes.fromhex(k) and int(dec["seqno"][i0 + j]) == s
            assert int(dec["handle_off"][i0 + j]) == o and int(dec["val_len"][i0 + j]) == z


def test_gpu_reference_hash_index_positions(gpu):
    """The reference's hash-index bytes (hash_index/mod.rs:48-79) pin
    bucket = hash64(key) % buckets: the GPU's xxh3_64 puts "a", "b", "c" in the
    buckets those bytes show."""
    import torch
    case = HASH["hash_index_build_simple"]
    keys = [bytes.fromhex(k) for k, _ in case["sets"]]
    kb, ko = _arena(keys)
    h = gpu.hash64_keys(gpu.to_device_bytes(kb), torch.from_numpy(ko).cuda())
    torch.cuda.synchronize()
    hv = h.cpu().numpy().view(np.uint64)
    for (k, idx), v in zip(case["sets"], hv):
        assert case["bytes"][int(v) % case["buckets"]] == idx


def test_gpu_reference_headers(gpu):
    """header.rs:177-214 on the device: the round-trip header passes its header
    checksum (then fails the payload checksum: the test header has no payload);
    the mutated one is a header checksum mismatch."""
    import torch
    blocks, want = [], []
    for name in sorted(HEADER):
        case = HEADER[name]
        hdr = bytearray(pyoracle.header_encode(case["block_type"], case["checksum"], case["data_length"],
                                               case["uncompressed_length"]))
        if case["mutate_byte"] is not None:
            hdr[case["mutate_byte"]] = (hdr[case["mutate_byte"]] + 1) & 0xFF
        blocks.append(bytes(hdr) + bytes(3))  # 16-B granule padding between the handles
        st, _ = pyoracle.block_verify(bytes(hdr))
        want.append(st)
    off = np.array([0, 33, 36, 69], np.int64)
    buf = blocks[0] + blocks[1]
    dec = gpu.decode_blocks(gpu.to_device_bytes(buf), torch.from_numpy(off).cuda(), 3)
    torch.cuda.synchronize()
    st = dec["status"][:3].cpu().numpy().tolist()
    assert st[0] == want[0] and st[2] == want[1]
    # sorted names: [block_header_detect_corruption, block_header_serde_roundtrip]
    assert want == [3, 4]  # HDR_CKSUM for the mutation; CKSUM for the round trip (the test header has no payload)
