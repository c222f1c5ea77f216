"""Every index a compiled image hands the kernels is in range (CPU).

The classify kernels trust the image: a cell's counter base plus a list
position (or a sublist state's slot field) indexes the slot counters, and
the finish launch maps a slot to its rule through ctr_rule
(vpp_amd/csrc/kernels_dev.hpp run_n, finish4_kernel; compile.hpp
Cls4Image).  A slot at or past n_ctr, or a rule past R, is a wild counter
write on the GPU.  The compiler builds the images in range by construction;
this test checks that independently of it: a static walk over each image as
the kernels read it (tests/cls_image.py's decoding) -- every cell of every
class and protocol, every port class, every state a sublist search can reach,
every source class a hash, interval or trie lookup can return -- on the
config 2, 3 and 5 tables and the gen-policy.py lists, both layouts.
"""
import random

import numpy as np
import pytest

from cls_image import Image, Image16, compile_blob
from vpp_amd import _abi

U32 = 0xFFFFFFFF


def _sublist_max_j(img, st0, steps):
    """Largest slot field ((state >> 2) & 63) over every state the sublist
    search (kernels: S probes, state >> 13 = entry byte address, entry
    {start - 1, state}) can reach from each initial state."""
    st0 = np.asarray(st0, np.int64)
    uniq, inv = np.unique(st0, return_inverse=True)
    origin = np.arange(len(uniq))
    st = uniq.copy()
    for i in range(int(steps) - 1, -1, -1):
        a = ((st >> 13) + (8 << i)) // 4
        assert (a >= 0).all() and (a + 1 < len(img)).all(), "sublist probe outside the image"
        key, nxt = img[a], img[a + 1]
        can = key != U32                       # some destination is above the key: the state moves
        origin = np.concatenate([origin, origin[can]])
        st = np.concatenate([st, nxt[can]])
        pair = np.unique(np.stack([origin, st], 1), axis=0)
        origin, st = pair[:, 0], pair[:, 1]
    mj = np.zeros(len(uniq), np.int64)
    np.maximum.at(mj, origin, (st >> 2) & 63)
    return mj[inv]


def _source_classes(im: Image):
    """Every class a source lookup of the image can return."""
    h = im.h
    img = np.frombuffer(im._img, np.uint32).astype(np.int64)
    if h.mode == 4:                            # trie: level 1 -> node -> leaves {key | class << 16}
        l1 = img[h.off_trie // 4 + np.arange(256)]
        node = img[(l1[:, None] + 4 * np.arange(256)[None, :]).ravel() // 4]
        node = np.unique(node)
        start, ln = node >> 8, (node & 0xFF) + 1
        idx = np.concatenate([s // 4 + np.arange(k) for s, k in zip(start, ln)])
        assert (idx < len(img)).all(), "trie leaf outside the image"
        return np.unique(img[idx] >> 16)
    if h.mode == 1:                            # hash LPM: entries {key, class row byte address}
        rows = [np.int64(h.default_row)]
        for _mask, _shift, _cap, tab, _mul in im.hash:
            rows.append(tab[:, 1].astype(np.int64))
        rows = np.unique(np.concatenate([np.atleast_1d(r) for r in rows]))
        assert ((rows - h.off_cells) % h.row_bytes == 0).all(), "hash row not a class row"
        return (rows - h.off_cells) // h.row_bytes
    if h.mode == 0:
        return np.unique(im.iclass[:h.n_bounds + 1].astype(np.int64)) if h.n_bounds else np.array([0])
    return np.arange(h.n_classes)             # mode 3: the caller's rows (checked by the front end)


def _port_classes4(im: Image):
    """Every port class x 4 of list modes 3-6 (all 65536 destination ports)."""
    return np.unique(im._port_class4(np.arange(65536, dtype=np.uint32)).astype(np.int64))


def check_image(im: Image, n_rules: int):
    h = im.h
    if not im.has_cls:
        return
    # slot -> rule (the finish launch's scatter): a rule of the table or its default DENY
    assert len(im.ctr_rule) == h.n_ctr
    assert (im.ctr_rule <= n_rules).all(), "slot mapped past the default DENY"
    assert h.n_hot <= max(h.n_lctr, h.n_hot) and h.n_lctr <= h.n_ctr
    assert h.n_ctr >= 1                        # slot 0: the no-match slot
    cls = _source_classes(im)
    assert (cls >= 0).all() and (cls < h.n_classes).all(), "source lookup returns a class past n_classes"
    img = np.frombuffer(im._img, np.uint32).astype(np.int64)
    cells = np.arange(h.n_classes)[:, None] * im.ncell + np.arange(im.ncell)[None, :]
    cells = cells.ravel()
    lm = h.list_mode
    if lm == 0:
        c = im.cells[cells].astype(np.int64)
        start, ln, base = c[:, 0] & 0xFFFF, c[:, 0] >> 16, c[:, 1]
        assert ((start + ln) <= h.n_list_entries).all(), "candidate list past the list table"
        assert (base + ln <= h.n_ctr).all(), "cell's slots past n_ctr (no match: slot 0)"
        assert (im.lists < h.n_tmpl).all(), "template id past n_tmpl"
    elif lm in (1, 2):
        c = img[h.off_cells // 4 + cells]
        d_off, cb = (c & 0xFFFF) * 2, c >> 16          # d table: 2^S {bound, mask} pairs (word offsets)
        S = int(h.bv_steps_d)
        win = d_off[:, None] + 2 * np.arange(1 << S)[None, :] + 1
        assert (win < len(img)).all(), "bit-vector table outside the image"
        masks = img[win]
        hib = np.zeros(len(c), np.int64)
        for b in range(31, -1, -1):               # highest bit over the whole window
            hit = ((masks >> b) & 1).any(1) & (hib == 0)
            hib[hit] = b
        live = masks.any(1)                       # an empty list never names a slot (no match: slot 0)
        assert (cb[live] + hib[live] < h.n_ctr).all(), "bit-vector slot past n_ctr"
    else:
        pc4 = _port_classes4(im)
        if lm >= 5:
            wc = im.gcells[cells].astype(np.int64)
            ptr, base = wc[:, 0], wc[:, 1]
        else:
            c = img[(h.off_cells + (cells // im.ncell) * h.row_bytes + (cells % im.ncell) * 4) // 4]
            ptr, base = (c & 0x3FFF) * 4, c >> 14
        a = (ptr[:, None] + pc4[None, :]) // 4
        assert (a < len(img)).all(), "pointer table outside the image"
        st0 = img[a]
        mj = _sublist_max_j(img, st0.ravel(), h.bv_steps_d).reshape(st0.shape)
        assert (base[:, None] + mj < h.n_ctr).all(), "sublist slot past n_ctr"
    if im.other is not None:
        check_image(im.other, n_rules)


def _v4(rules):
    return Image(compile_blob(_abi.CRules(rules)))


def _v16(rules):
    return Image16(compile_blob(_abi.CRules(rules), "cls_compile_v16"))


@pytest.mark.parametrize("cfg", [2, 3, 5])
def test_config_tables_in_range(cfg):
    from vpp_amd import workload
    acl, _spec, _ = workload.config(cfg)
    n = len(acl.rules)
    if cfg != 5:
        im = _v4(acl.rules)
        assert im.has_cls
        check_image(im, n)
    im16 = _v16(acl.rules)
    assert im16.core.has_cls
    check_image(im16.core, n)
    h = im16.h
    if h.src_mode == 1:                        # host-route hashes: rows of the core
        rows = np.array([h.dflt_row[0], h.dflt_row[1]], np.int64)
        assert ((rows - im16.core.h.off_cells) // im16.core.h.row_bytes < im16.core.h.n_classes).all()


def _gen_policy_list(blocks, match):
    from vpp_amd import configurator as C
    from vpp_amd.renderer.api import PodID
    from vpp_amd.renderer.traffic import compile_rules
    pol = C.gen_policy(random.Random(blocks), num_cidrs=blocks)
    txn = C.PolicyConfigurator({PodID("db", "default"): "10.1.1.1"}).new_txn(False)
    return compile_rules(txn.generate_rules(match, [pol]))


@pytest.mark.parametrize("blocks", [20, 200, 1000])
@pytest.mark.parametrize("match", ["ingress", "egress"])
def test_gen_policy_lists_in_range(blocks, match):
    from vpp_amd import configurator as C
    rules = _gen_policy_list(blocks, {"ingress": C.MATCH_INGRESS, "egress": C.MATCH_EGRESS}[match])
    check_image(_v4(rules), len(rules))
    check_image(_v16(rules).core, len(rules))


@pytest.mark.parametrize("seed", range(6))
def test_random_acls_every_list_mode_in_range(seed, libopt):
    """Random ACLs with malformed rules under every list-mode cap and source
    lookup (hash, interval search, trie)."""
    from aclgen import long_list_acl, many_ports_acl, random_acl, single_port_acl
    gens = [random_acl(seed, 300, 0.1), single_port_acl(seed + 3, 200), many_ports_acl(seed, 300, 30),
            long_list_acl(seed + 1, 250)]
    for rules, _pool in gens:
        for cap in (0, 1, 2, 3, 4, 6):
            for trie in ("0", "1"):
                libopt.set("list_mode_max", cap)
                libopt.set("trie", trie)
                check_image(_v4(rules), len(rules))
