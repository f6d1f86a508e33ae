"""The literal DPDK 17.11 rte_lpm (v1604) restatement (oracle/dpdk_lpm_v1604.c:
rules_tbl grouped by depth with rule_info[depth-1] = {used_rules, first_rule},
rule_add_v1604 / rule_delete_v1604, tbl8_alloc_v1604) against the oracle's
hash-based restatement (cop_oracle.c orc_lpm_*) and the product's builder
(csrc/lpm_build.c, cop_lpm_build), on add sequences that interleave tbl8
exhaustion, max_rules exhaustion, duplicate (prefix, depth) updates and
invalid depths, in lpm_setup's stop-at-first-error mode (firewall.c:243-252)
and in continue-on-error mode.

Compared: every add's return code, the accepted rule set, tbl8 groups in
use, and the lookup of every probe address (both device images of the
product). DPDK itself is not available here, so this pins the product to
two independent restatements of DPDK's published algorithm, not to DPDK's
own outputs (parity unpinned against the reference)."""
import numpy as np
import pytest

import copgpu as cg
import oracle as orc
from test_lpm_host import lookup_dir24, lookup_intervals, probes_for


def rule_mix(rng, n, n_parents, max_depth_small=24):
    """n rules: ~40 % depth 25..32 spread over n_parents /24s (tbl8 groups),
    the rest depth 1..24, ~15 % repeats of earlier (prefix, depth) with new
    next hops, ~2 % invalid depths."""
    parents = rng.integers(0, 1 << 24, n_parents, dtype=np.uint64).astype(np.uint32)
    ip = np.zeros(n, np.uint32)
    d = np.zeros(n, np.uint8)
    nh = rng.integers(0, 1 << 24, n, dtype=np.uint64).astype(np.uint32)
    for i in range(n):
        u = rng.random()
        if i > 4 and u < 0.15:
            k = int(rng.integers(0, i))
            ip[i], d[i] = ip[k], d[k]
        elif u < 0.17:
            ip[i] = int(rng.integers(0, 2**32))
            d[i] = int(rng.choice([0, 33, 40]))
        elif u < 0.57:
            p = parents[int(rng.integers(0, n_parents))]
            ip[i] = (int(p) << 8) | int(rng.integers(0, 256))
            d[i] = int(rng.integers(25, 33))
        else:
            ip[i] = int(rng.integers(0, 2**32))
            d[i] = int(rng.integers(1, max_depth_small + 1))
    return cg.prefixes(ip, d, nh)


def check_rule_info(dl):
    """rules_tbl invariants: non-empty groups are contiguous, in depth
    order, cover [0, n_rules)."""
    used, first = dl.rule_info()
    pos = 0
    for dep in range(32):
        if used[dep]:
            assert first[dep] == pos, (dep, first[dep], pos)
            pos += used[dep]
    assert pos == dl.n_rules


def compare_all(rules, max_rules, ntbl8, stop, rng):
    dl = orc.DpdkLpm(max_rules, ntbl8)
    first_dl, err_dl, rc_dl = dl.setup(rules["ip"], rules["depth"], rules["next_hop"], stop_at_error=stop)
    check_rule_info(dl)
    # the hash restatement, add by add
    o = orc.OracleLpm(max_rules, ntbl8)
    rc_o = []
    for i, (ip, dep, nh) in enumerate(zip(rules["ip"], rules["depth"], rules["next_hop"])):
        r = o.add(int(ip), int(dep), int(nh))
        rc_o.append(r)
        if r < 0 and stop:
            rc_o += [-9999] * (len(rules) - i - 1)
            break
    assert list(rc_dl) == rc_o
    assert dl.n_rules == o.n_rules and dl.tbl8_used == o.tbl8_used
    # the product's builder
    t = cg.LpmTable(rules, max_rules, ntbl8, stop)
    rep = t.report
    presented = rc_dl[rc_dl != -9999]
    assert rep.n_failed == int(np.sum(presented < 0))
    assert rep.n_skipped == int(np.sum(rc_dl == -9999))
    assert rep.first_error_idx == (first_dl if first_dl >= 0 else rep.first_error_idx)
    assert rep.first_error == err_dl
    assert rep.n_distinct == dl.n_rules and rep.tbl8_used == dl.tbl8_used
    # rule sets (DPDK keeps them grouped by depth; compare as sets)
    dip, dd, dnh = dl.rules()
    pr = t.rules()
    a = sorted(zip(dip.tolist(), dd.tolist(), dnh.tolist()))
    b = sorted(zip(pr["ip"].tolist(), pr["depth"].tolist(), pr["next_hop"].tolist()))
    assert a == b
    # lookups: literal == hash restatement == both product images
    ips = probes_for(rules[(rules["depth"] >= 1) & (rules["depth"] <= 32)], rng, 20000)
    dnh_, dhit = dl.lookup(ips)
    onh, ohit = o.lookup(ips)
    assert np.array_equal(dnh_, onh) and np.array_equal(dhit, ohit)
    for fn in (lookup_intervals, lookup_dir24):
        nh, hit = fn(t, ips)
        assert np.array_equal(nh, dnh_), fn.__name__
        assert np.array_equal(hit, dhit), fn.__name__
    return dl, rc_dl


@pytest.mark.parametrize("seed", range(6))
@pytest.mark.parametrize("stop", [True, False])
def test_interleaved_exhaustion(seed, stop):
    """max_rules and tbl8 groups both run out, in either order, with updates
    and invalid depths in between."""
    rng = np.random.default_rng(seed)
    max_rules, ntbl8 = int(rng.integers(24, 96)), int(rng.integers(1, 6))
    rules = rule_mix(rng, 400, n_parents=ntbl8 + 4)
    dl, rc = compare_all(rules, max_rules, ntbl8, stop, rng)
    if not stop:
        assert np.sum(rc == -28) > 0          # -ENOSPC happened and loading continued
        assert np.sum(rc == 0) > 0


def test_reference_limits_fw_rule_files():
    """lpm_setup's own limits (1024 rules, 24 tbl8 groups) on rule files
    bigger than both, stop-at-first-error as firewall.c:245-251."""
    rng = np.random.default_rng(42)
    for seed in (1, 2):
        rules = cg.gen_rules(seed, 3000, cg.GEN_FW, 60)
        compare_all(rules, 1024, 24, True, rng)
        compare_all(rules, 1024, 24, False, rng)


def test_stale_first_rule_of_an_empty_group():
    """rule_add_v1604 sets an empty group's first_rule before it checks the
    deeper groups for room: a -ENOSPC there leaves the stale first_rule in
    rule_info. It is never read while the group is empty; later updates,
    refusals and lookups are unaffected."""
    dl = orc.DpdkLpm(2, 4)
    assert dl.add(0x0A000001, 32, 1) == 0
    assert dl.add(0x0A000002, 32, 2) == 0               # group 32 fills rules_tbl [0, 2)
    assert dl.add(0x0B000000, 16, 3) == -28             # no room: -ENOSPC
    used, first = dl.rule_info()
    assert used[15] == 0 and first[15] == 0 and used[31] == 2   # the stale first_rule
    assert dl.add(0x0A000001, 32, 9) == 0               # an update still succeeds
    assert dl.add(0x0C000000, 8, 4) == -28
    nh, hit = dl.lookup(np.array([0x0A000001, 0x0A000002, 0x0B000000], np.uint32))
    assert list(nh) == [9, 2, 0] and list(hit) == [1, 1, 0]
    rules = cg.prefixes([0x0A000001, 0x0A000002, 0x0B000000, 0x0A000001, 0x0C000000], [32, 32, 16, 32, 8],
                        [1, 2, 3, 9, 4])
    compare_all(rules, 2, 4, False, np.random.default_rng(0))


def test_tbl8_failure_deletes_the_new_rule():
    """A depth > 24 rule that needs a tbl8 group when none is free fails
    with -ENOSPC and rule_delete_v1604 takes it back out of rules_tbl; the
    deeper groups shifted for it move back."""
    dl = orc.DpdkLpm(16, 1)
    assert dl.add(0x0A000080, 25, 1) == 0               # takes the only group
    assert dl.add(0x0A000000, 30, 2) == 0               # same /24: no new group
    assert dl.add(0x14000000, 28, 5) == -28             # another /24: no group left
    assert dl.n_rules == 2 and dl.tbl8_used == 1
    check_rule_info(dl)
    assert dl.add(0x0B000000, 8, 3) == 0                # shifts groups 25 and 30 up
    assert dl.add(0x15000000, 26, 6) == -28             # fails again, groups shift back
    check_rule_info(dl)
    ip, d, nh = dl.rules()
    assert list(d) == [8, 25, 30] and list(nh) == [3, 1, 2]
