"""Device materialize (lsm_materialize_plan / lsm_materialize_keys) ==
DataBlockParsedItem::materialize (src/table/data_block/mod.rs:296-315) as restated by
pyoracle.materialize: every key = Slice::fused(restart-head prefix, suffix), values as
(val_off, val_len) sub-slices.  Blocks cover restart intervals 1..64, prefix-heavy keys,
tombstones, index blocks (end keys, no prefix) and a corrupt block (empty keys)."""
import numpy as np
import pytest

from helpers import counter_items, index_items, pack, prefix_items, random_sorted_items

pytestmark = pytest.mark.gpu


def _blocks(oracle):
    blocks, ris = [], []
    for s, ri in enumerate([1, 2, 3, 5, 16, 64]):
        items = random_sorted_items(150, seed=s, kmax=40)
        blocks.append(oracle.block_write(oracle.data_block_encode(items, restart_interval=ri)))
        ris.append(ri)
    blocks.append(oracle.block_write(oracle.data_block_encode(prefix_items(56, seed=2))))
    blocks.append(oracle.block_write(oracle.data_block_encode(counter_items(820, seed=3, tomb_frac=0.1))))
    blocks.append(oracle.block_write(oracle.index_block_encode(index_items(40)), block_type=1))
    return blocks


def test_materialize_keys_match_oracle(gpu, oracle):
    import torch
    blocks = _blocks(oracle)
    bad = bytearray(blocks[2])
    bad[50] ^= 0x10  # checksum mismatch: the block's items get empty keys
    blocks[2] = bytes(bad)
    buf, off = pack(blocks)
    d_blocks = gpu.to_device_bytes(buf)
    d_off = torch.from_numpy(off.astype(np.int64)).cuda()
    n = len(blocks)
    out = gpu.decode_blocks(d_blocks, d_off, n)
    keys, key_off = gpu.materialize_keys(d_blocks, d_off, n, out)
    torch.cuda.synchronize()
    st = out["status"].cpu().numpy()[:n]
    assert st[2] == 4 and (np.delete(st, 2) == 0).all()
    item_start = out["item_start"].cpu().numpy().view(np.uint32)
    ko = key_off.cpu().numpy()
    kb = keys.cpu().numpy().tobytes()
    parsed_all = {f: out[f].cpu().numpy() for f in ("seqno", "key_off", "key_len", "prefix_len", "val_off", "val_len",
                                                    "vtype")}
    for b in range(n):
        lo, hi = int(item_start[b]), int(item_start[b + 1])
        if st[b] != 0:
            assert (ko[lo:hi + 1] == ko[lo]).all()  # empty keys
            continue
        payload = bytes(buf[int(off[b]) + 33:int(off[b + 1])])
        cnt, parsed = oracle.data_block_decode(payload, index=(b == n - 1))
        assert cnt == hi - lo
        ri = payload[-31]
        want = oracle.materialize(payload, parsed, ri)
        for k, (key, val, seq, vt) in enumerate(want):
            i = lo + k
            assert kb[ko[i]:ko[i + 1]] == key, (b, k)
            vo, vl = int(parsed_all["val_off"][i]), int(parsed_all["val_len"][i])
            if b != n - 1:  # index blocks: val_len is the handle size, not a value
                assert payload[vo:vo + vl] == val and int(parsed_all["vtype"][i]) == vt


def test_scan_then_materialize(gpu, oracle):
    """Scanner + materialize: the scanned table's keys are the written keys."""
    import torch
    items = random_sorted_items(2000, seed=11, kmax=30)
    t = oracle.table_write(items, two_level=True, block_size=512)
    d_file = gpu.to_device_bytes(t["file"])
    out = gpu.scan_table(d_file, len(t["file"]), t["tli_off"], t["tli_size"], two_level=True,
                         block_count=t["block_count"])
    assert out["table_status"] == 0
    nb = out["n_blocks"]
    keys, key_off = gpu.materialize_keys(d_file, out["block_off"], nb, out)
    torch.cuda.synchronize()
    ko = key_off.cpu().numpy()
    kb = keys.cpu().numpy().tobytes()
    want = [items.keys[int(items.key_off[i]):int(items.key_off[i + 1])].tobytes() for i in range(items.n)]
    assert len(ko) == items.n + 1
    assert [kb[ko[i]:ko[i + 1]] for i in range(items.n)] == want


def test_materialize_output_past_2gib(gpu):
    """A key arena larger than 2 GiB (1000-byte keys: 992-byte shared prefix +
    8-byte counter, restart interval 16): output offsets with bit 31 set must
    not be sign-extended when a wave broadcasts them (the v_readfirstlane int
    result is widened through uint32_t).  Every materialized key equals the
    encoder's input key."""
    import sys
    from pathlib import Path
    import torch
    sys.path.insert(0, str(Path(__file__).resolve().parent.parent))
    import bench
    n_blocks = 520000  # 5 items of 1000 + 4 bytes per 4 KiB block: 2.6 M keys, 2.6 GB materialized
    items, starts, n = bench.make_workload(torch, gpu, n_blocks, items_per_block=5, key_len=1000, val_len=4,
                                           seed=77, kind="prefix")
    bench.check_cut_rule(gpu, 5, 1000, 4)
    enc = gpu.Encoder().encode(items, starts, n_blocks)
    torch.cuda.synchronize()
    assert int((enc["status"][:n_blocks] != 0).sum()) == 0
    out = gpu.decode_blocks(enc["buf"], enc["block_off"], n_blocks, item_cap=n)
    keys, key_off = gpu.materialize_keys(enc["buf"], enc["block_off"], n_blocks, out, n)
    torch.cuda.synchronize()
    assert int((out["status"][:n_blocks] != 0).sum()) == 0
    assert int(key_off[n].item()) == n * 1000 and n * 1000 > (1 << 31) + (1 << 28)
    assert torch.equal(key_off[:n + 1], torch.arange(n + 1, device=key_off.device, dtype=key_off.dtype) * 1000)
    assert torch.equal(keys[:n * 1000], items["keys"][:n * 1000])


def test_materialize_capped_no_sync(gpu, oracle):
    """lsm_materialize_keys_capped: an arena sized without reading the plan back.
    Large enough: the keys and offsets equal the two-call path's (items past
    item_start[n_blocks], up to the parsed arrays' capacity, get empty keys);
    one byte short: LSM_OVERFLOW on the device and nothing written."""
    import torch
    blocks = _blocks(oracle)
    buf, off = pack(blocks)
    d_blocks = gpu.to_device_bytes(buf)
    d_off = torch.from_numpy(off.astype(np.int64)).cuda()
    n = len(blocks)
    out = gpu.decode_blocks(d_blocks, d_off, n)
    keys, key_off = gpu.materialize_keys(d_blocks, d_off, n, out)
    torch.cuda.synchronize()
    total = int(key_off[-1].item())
    n_items = key_off.numel() - 1
    k2, o2, res = gpu.materialize_keys(d_blocks, d_off, n, out, key_cap=total)
    torch.cuda.synchronize()
    assert int(res.item()) == 0
    assert o2.numel() == out["key_off"].numel() + 1
    assert torch.equal(o2[:n_items + 1], key_off) and (o2[n_items:] == total).all()
    assert torch.equal(k2[:total], keys[:total])
    k3, o3, res3 = gpu.materialize_keys(d_blocks, d_off, n, out, key_cap=total - 1)
    torch.cuda.synchronize()
    assert int(res3.item()) == 6  # LSM_OVERFLOW
    assert int((k3[:total - 1] != 0).sum().item()) == 0  # (padded_bytes zero-fills; nothing written)
