"""ISA check of tools/micro/issue_cost.hip: every k_issue<K> loop body holds exactly the
instructions the kind promises (16 of its class, or the mix), and no other vector
instruction, so the wall-clock costs are per-class issue costs (not collapsed, not diluted).

usage: python tools/micro/issue_cost_check.py ISSUE_COST.s
Prints one line per kind and exits non-zero on a mismatch.
"""
import collections
import re
import sys

# kind -> {opcode prefix: count per loop iteration}
EXPECT = {
    0: {"v_fma_f64": 16}, 1: {"v_mul_f64": 16}, 2: {"v_add_f64": 16}, 3: {"v_fma_f32": 16},
    4: {"v_mul_f32": 16}, 5: {"v_pk_fma_f32": 16}, 6: {"v_pk_mul_f32": 16}, 7: {"v_add_u32": 16},
    8: {"v_and_b32": 16}, 9: {"v_lshl_add_u32": 16}, 10: {"v_mov_b32": 16}, 11: {"v_mov_b64": 16},
    12: {"v_cndmask_b32": 16}, 13: {"v_cmp_lt_f32": 16}, 14: {"v_cmp_lt_f64": 16}, 15: {"v_mad_u64_u32": 16},
    16: {"v_lshl_add_u64": 16}, 17: {"v_cvt_f32_f64": 16}, 18: {"v_rsq_f32": 16},
    19: {"v_fma_f64": 16, "v_pk_fma_f32": 32}, 20: {"v_pk_fma_f32": 16, "v_add_u32": 16},
    21: {"s_add_u32": 16}, 22: {"v_pk_fma_f32": 16, "s_add_u32": 16}, 23: {"v_pk_fma_f32": 16, "s_add_u32": 8},
    24: {"v_pk_fma_f32": 16, "ds_read_b64": 8}, 25: {"v_pk_fma_f32": 16, "v_cmp_lt_f32": 16},
}
for _k, _op in enumerate(["v_fmac_f32_e32", "v_add_f32_e32", "v_cmp_lt_f32_e32", "v_cndmask_b32_e32", "v_or3_b32",
                          "v_pk_add_f32", "v_max_f32_e32", "v_readfirstlane_b32", "v_fmac_f64_e32",
                          "v_mbcnt_lo_u32_b32", "v_lshlrev_b64", "v_bfe_u32", "v_cvt_f64_f32"], start=26):
    EXPECT[_k] = {_op: 16}
EXPECT.update({39: {"v_fma_f32": 16}, 40: {"v_fma_f32": 16}, 41: {"v_pk_fma_f32": 16}, 42: {"v_pk_fma_f32": 16},
               43: {"v_fma_f64": 16}, 44: {"v_pk_fma_f32": 16, "s_cselect_b64": 16, "s_andn2_b64": 16, "s_cmp_lg_u32": 16}})
# non-vector instructions counted for the kinds that promise them
COUNTED = ("s_add_u32", "ds_read_b64", "s_cselect_b64", "s_andn2_b64", "s_cmp_lg_u32")


def loop_body(asm: str, kind: int) -> list:
    m = re.search(r"^(_Z\w*k_issueILi%dE\w*):" % kind, asm, re.M)
    if not m:
        raise SystemExit(f"kind {kind}: kernel not found")
    body = asm[m.end(): asm.find(".Lfunc_end", m.end())]
    # the loop: the basic block that ends with a backward conditional branch to its own label
    blocks = re.split(r"^(\.LBB\w+):", body, flags=re.M)
    for i in range(1, len(blocks), 2):
        label, text = blocks[i], blocks[i + 1]
        br = re.search(r"s_cbranch_\w+\s+%s\b" % re.escape(label), text)
        if br:
            return [ln.split()[0] for ln in text[: br.end()].splitlines()
                    if ln.strip() and not ln.strip().startswith((";", "."))]
    raise SystemExit(f"kind {kind}: loop not found")


def main():
    asm = open(sys.argv[1]).read()
    bad = 0
    for kind, want in EXPECT.items():
        ops = loop_body(asm, kind)
        vec = collections.Counter(o for o in ops if o.startswith("v_") or o.startswith(COUNTED))
        got = {k: sum(v for o, v in vec.items() if o.startswith(k)) for k in want}
        other = {o: v for o, v in vec.items() if not any(o.startswith(k) for k in want)}
        ok = got == want and not other
        bad += not ok
        print(f"kind {kind:2d} {'ok ' if ok else 'BAD'} loop VALU {dict(vec)}"
              + ("" if ok else f" want {want} other {other}"))
    sys.exit(1 if bad else 0)


if __name__ == "__main__":
    main()
