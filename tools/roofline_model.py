"""VALU-issue roofline model of one kernel: per-class instruction counts x measured issue costs.

Counts: the PMC class counters of the kernel (SQ_INSTS_VALU_{FMA,MUL,ADD,TRANS}_F32/F64,
_INT32, _INT64, _CVT, and SQ_INSTS_VALU for the rest), per dispatch, from a committed summary
(tools/valu_class_pmc.py). Which opcode each counter counts was calibrated on the
micro-benchmark (profiles/r03_issue_cost_pmc.json: v_pk_fma_f32 and v_fma_f32 both count in
FMA_F32, v_add_u32 and v_lshl_add_u32 in INT32, compares / moves / selects / bit ops in none).
Inside one counter class, the opcodes are split in the proportions of the kernel's own ISA
(hipcc --cuda-device-only -S of the same source; each opcode weighted by its static count),
and the instructions no class counter sees (SQ_INSTS_VALU minus the classes) in the
proportions of the ISA's unclassified opcodes.
Costs: SIMD-cycles per wave64 instruction measured at wall clock by tools/micro/issue_cost.hip
at the kernel's waves per SIMD (profiles/r03_issue_cost.json, ISA-checked loop bodies); opcodes
not measured take the cost of the measured opcode of the same encoding class (rules below).

cycles = sum_class count_class x (ISA-weighted mean cost of the class's opcodes)
frac   = cycles / (1024 SIMDs x 2.4e9 x kernel time)   (bench.py divides by the live time)
Also reported: the same with every class at its cheapest / dearest member (bounds on the
split), and the SALU instructions' marginal issue cost measured beside packed FMAs.

usage: python tools/roofline_model.py ISA.s KERNEL_SUBSTR PMC.json PMC_KERNEL_NAME COSTS.json WAVES OUT.json
"""
import collections
import json
import re
import sys

# PMC class of an opcode (calibrated; None = no class counter counts it)
CLASS_RULES = [
    (r"^v_pk_fma_f32|^v_fma_f32|^v_fmac_f32|^v_fmamk_f32|^v_fmaak_f32", "FMA_F32"),
    (r"^v_pk_mul_f32|^v_mul_f32", "MUL_F32"),
    (r"^v_pk_add_f32|^v_add_f32|^v_sub_f32|^v_subrev_f32", "ADD_F32"),
    (r"^v_(rcp|rsq|sqrt|exp|log|sin|cos)_f32", "TRANS_F32"),
    (r"^v_fma_f64|^v_fmac_f64", "FMA_F64"),
    (r"^v_mul_f64", "MUL_F64"),
    (r"^v_add_f64", "ADD_F64"),
    (r"^v_(rcp|rsq|sqrt)_f64", "TRANS_F64"),
    (r"^v_mad_u64_u32|^v_lshl_add_u64|^v_mad_i64_i32", "INT64"),
    (r"^v_add_u32|^v_sub_u32|^v_subrev_u32|^v_lshl_add_u32|^v_add_lshl_u32|^v_mul_lo_u32|^v_mad_u32_u24|^v_add3_u32", "INT32"),
    (r"^v_cvt_", "CVT"),
]
PMC_OF = {"FMA_F32": "SQ_INSTS_VALU_FMA_F32", "MUL_F32": "SQ_INSTS_VALU_MUL_F32", "ADD_F32": "SQ_INSTS_VALU_ADD_F32",
          "TRANS_F32": "SQ_INSTS_VALU_TRANS_F32", "FMA_F64": "SQ_INSTS_VALU_FMA_F64", "MUL_F64": "SQ_INSTS_VALU_MUL_F64",
          "ADD_F64": "SQ_INSTS_VALU_ADD_F64", "TRANS_F64": "SQ_INSTS_VALU_TRANS_F64", "INT32": "SQ_INSTS_VALU_INT32",
          "INT64": "SQ_INSTS_VALU_INT64", "CVT": "SQ_INSTS_VALU_CVT"}

# cost key (a measured micro-benchmark row) of an opcode: exact name first, then encoding rules
COST_RULES = [
    (r"^v_pk_", "v_pk_fma_f32"),
    (r"^v_(fma|fmac)_f64", "v_fma_f64"),
    (r"^v_mul_f64", "v_mul_f64"),
    (r"^v_(add|min|max|ldexp|frexp_mant|fract|trig_preop|div_fixup|div_fmas|div_scale)_f64|^v_(max|min)_f64", "v_add_f64"),
    (r"^v_(rcp|rsq|sqrt)_f64", "v_rsq_f32x2"),
    (r"^v_(rcp|rsq|sqrt|exp|log|sin|cos)_f32", "v_rsq_f32"),
    (r"^v_fmac_f32_e32", "v_fmac_f32_e32"),
    (r"^v_(fma|fmamk|fmaak)_f32", "v_fma_f32"),
    (r"^v_cmp.*_e32$|^v_cmpx.*_e32$", "v_cmp_lt_f32_e32"),
    (r"^v_cmp", "v_cmp_lt_f32"),
    (r"^v_cndmask", "v_cndmask_b32"),      # the e32 (VCC) row of the micro-benchmark is an outlier
    (r"^v_readlane|^v_readfirstlane|^v_writelane", "v_readfirstlane_b32"),
    (r"^v_mov_b64|^v_lshlrev_b64|^v_lshrrev_b64|^v_ashrrev_i64|.*_u64|.*_i64|.*_b64", "v_mov_b64"),
    (r"^v_cvt_f64", "v_cvt_f64_f32"),
    (r"^v_cvt", "v_cvt_f32_f64"),
    (r"^v_accvgpr_(read|write|mov)", "v_mov_b32"),
    # 32-bit VOP2 (e32) forms: one or two sources, the cheap issue class
    (r"^v_\w+_e32$", "v_add_u32"),
    (r"^v_(mov|not)_b32", "v_mov_b32"),
    (r"^v_(and|or|xor)_b32$|^v_(add|sub|subrev)_u32$|^v_(lshlrev|lshrrev|ashrrev)_b32$", "v_add_u32"),
    # everything else: VOP3 (three sources or an e64 modifier form)
    (r"^v_", "v_lshl_add_u32"),
]
SKIP = re.compile(r"^v_nop|^v_mfma|^v_smfmac")


def isa_opcodes(path, pat):
    s = open(path).read()
    m = re.search(r"^(_Z[^ :]*%s[^ :]*):" % re.escape(pat), s, re.M)
    body = s[m.start(): s.find(".Lfunc_end", m.start())]
    cnt = collections.Counter()
    for line in body.splitlines():
        t = line.strip().split()
        if t and t[0].startswith("v_") and not SKIP.match(t[0]):
            cnt[t[0]] += 1
    return cnt


def class_of(op):
    for rx, c in CLASS_RULES:
        if re.match(rx, op):
            return c
    return None


def cost_of(op, costs):
    base = op
    if base in costs:
        return costs[base], base
    stem = re.sub(r"_e(32|64)$", "", op)
    if stem in costs and not op.endswith("_e32"):
        return costs[stem], stem
    for rx, key in COST_RULES:
        if re.match(rx, op):
            if key == "v_rsq_f32x2":
                return 2.0 * costs["v_rsq_f32"], key
            return costs[key], key
    raise KeyError(op)


def class_cycles(ops, pmc, costs, sub=None):
    """cycles of one region: per class, the region's dynamic count (pmc minus `sub` when given)
    times the mean cost of the class's opcodes in the region's static mix"""
    by_class = collections.defaultdict(dict)
    for op, n in ops.items():
        if n > 0:
            by_class[class_of(op) or "OTHER"][op] = n
    dyn = dict(pmc)
    if sub is not None:
        dyn = {k: max(pmc.get(k, 0.0) - sub.get(k, 0.0), 0.0) for k in set(pmc) | set(sub)}
    total = dyn.get("SQ_INSTS_VALU", 0.0)
    counted, cyc, lo, hi, detail = 0.0, 0.0, 0.0, 0.0, {}
    for cls, members in sorted(by_class.items()):
        n_dyn = (total - sum(dyn.get(PMC_OF[c], 0.0) for c in PMC_OF)) if cls == "OTHER" else dyn.get(PMC_OF[cls], 0.0)
        n_dyn = max(n_dyn, 0.0)
        counted += n_dyn
        static = sum(members.values())
        cs = {op: cost_of(op, costs) for op in members}
        mean = sum(members[op] * cs[op][0] for op in members) / static
        cyc += n_dyn * mean
        lo += n_dyn * min(c for c, _ in cs.values())
        hi += n_dyn * max(c for c, _ in cs.values())
        detail[cls] = {"dynamic": n_dyn, "mean_cost": mean, "isa_static": dict(members)}
    return {"valu_instructions": total, "valu_issue_cycles": cyc, "bounds": [lo, hi], "classes": detail,
            "salu_instructions": dyn.get("SQ_INSTS_SALU", 0.0)}


def main_regions():
    """Two-region form (round 4): the dominant kernel's dynamic class counts split into its y
    sweep and everything else by an ablation build without the sweeps (-DPCG_TGF_ABL=1): sweep =
    base PMC - ablation PMC, rest = ablation PMC, each class's opcodes weighted by that region's
    own static mix (sweep = the opcodes the base ISA has beyond the ablation ISA; rest = the
    ablation ISA). usage: roofline_model.py --regions BASE.s ABL.s KERNEL_SUBSTR PMC_BASE.json
    PMC_ABL.json PMC_KERNEL_NAME COSTS.json WAVES OUT.json"""
    a = sys.argv[sys.argv.index("--regions") + 1:]
    isa_b, isa_a, pat, pmcb, pmca, pmck, costf, waves, out = a[:9]
    waves = int(waves)
    rows = json.load(open(costf))["rows"]
    costs = {r["name"].split(" ")[0]: r["cyc_at_2p4"] for r in rows if r["waves_per_simd"] == waves
             and not r["name"].startswith("mix") and "bank" not in r["name"]}
    costs.pop("v_cndmask_b32_e32", None)
    ob, oa = isa_opcodes(isa_b, pat), isa_opcodes(isa_a, pat)
    sweep_ops = collections.Counter({op: ob[op] - oa.get(op, 0) for op in ob if ob[op] > oa.get(op, 0)})
    pb = {k: v["per_dispatch_mean"] for k, v in json.load(open(pmcb))[pmck].items()}
    pa = {k: v["per_dispatch_mean"] for k, v in json.load(open(pmca))[pmck].items()}
    sweep = class_cycles(sweep_ops, pb, costs, sub=pa)
    rest = class_cycles(oa, pa, costs)
    total = pb["SQ_INSTS_VALU"]
    cyc = sweep["valu_issue_cycles"] + rest["valu_issue_cycles"]
    res = {"kernel": pmck, "waves_per_simd": waves, "model": "two-region dynamic (sweep / rest by ablation build)",
           "valu_instructions": total, "valu_issue_cycles": cyc,
           "valu_issue_cycles_bounds": [sweep["bounds"][0] + rest["bounds"][0], sweep["bounds"][1] + rest["bounds"][1]],
           "mean_cycles_per_valu": cyc / total, "salu_instructions": pb.get("SQ_INSTS_SALU", 0.0),
           "regions": {"sweep": sweep, "rest": rest}, "cost_source": costf,
           "pmc_source": [pmcb, pmca], "isa_source": [isa_b, isa_a]}
    json.dump(res, open(out, "w"), indent=1, sort_keys=True)
    print(json.dumps({k: res[k] for k in ("kernel", "valu_instructions", "valu_issue_cycles", "valu_issue_cycles_bounds",
                                          "mean_cycles_per_valu")}))
    print("sweep", round(sweep["valu_instructions"]), round(sweep["valu_issue_cycles"]), "rest",
          round(rest["valu_instructions"]), round(rest["valu_issue_cycles"]))


def main():
    if "--regions" in sys.argv:
        return main_regions()
    isa, pat, pmcf, pmck, costf, waves, out = sys.argv[1:8]
    waves = int(waves)
    rows = json.load(open(costf))["rows"]
    costs = {r["name"]: r["cyc_at_2p4"] for r in rows if r["waves_per_simd"] == waves and not r["name"].startswith("mix")
             and "bank" not in r["name"]}
    costs = {k.split(" ")[0]: v for k, v in costs.items()}
    # the VCC-sourced select row (v_cndmask_b32_e32, ~23 cycles at every occupancy) is an outlier
    # of that micro-benchmark kernel (no VCC write in its loop), not a property of the kernels
    # modelled here: their selects take the measured e64 cost
    costs.pop("v_cndmask_b32_e32", None)
    mix = {r["name"]: r["cyc_at_2p4"] for r in rows if r["waves_per_simd"] == waves and r["name"].startswith("mix")}
    ops = isa_opcodes(isa, pat)
    pmc = {k: v["per_dispatch_mean"] for k, v in json.load(open(pmcf))[pmck].items()}
    by_class = collections.defaultdict(dict)
    for op, n in ops.items():
        by_class[class_of(op) or "OTHER"][op] = n
    total = pmc["SQ_INSTS_VALU"]
    counted = 0.0
    detail, cyc, lo, hi = {}, 0.0, 0.0, 0.0
    for cls, members in sorted(by_class.items()):
        if cls == "OTHER":
            continue
        n_dyn = pmc.get(PMC_OF[cls], 0.0)
        counted += n_dyn
        static = sum(members.values())
        cs = {op: cost_of(op, costs) for op in members}
        mean = sum(members[op] * cs[op][0] for op in members) / static
        cyc += n_dyn * mean
        lo += n_dyn * min(c for c, _ in cs.values())
        hi += n_dyn * max(c for c, _ in cs.values())
        detail[cls] = {"dynamic": n_dyn, "mean_cost": mean, "isa_static": dict(members),
                       "costs": {op: [round(c, 3), k] for op, (c, k) in cs.items()}}
    other = max(total - counted, 0.0)
    members = by_class.get("OTHER", {})
    if members:
        static = sum(members.values())
        cs = {op: cost_of(op, costs) for op in members}
        mean = sum(members[op] * cs[op][0] for op in members) / static
        cyc += other * mean
        lo += other * min(c for c, _ in cs.values())
        hi += other * max(c for c, _ in cs.values())
        detail["OTHER (no class counter)"] = {"dynamic": other, "mean_cost": mean, "isa_static": dict(members),
                                              "costs": {op: [round(c, 3), k] for op, (c, k) in cs.items()}}
    salu = pmc.get("SQ_INSTS_SALU", 0.0)
    # marginal SALU cost next to packed FMAs (one wave's interleaved stream, same waves/SIMD):
    # (mix cycles x its instruction count - the FMAs' own cycles) / SALU count
    pk = costs["v_pk_fma_f32"]
    m1 = mix.get("mix:pk_fma_f32+s_add_u32")
    m3 = mix.get("mix:pk_fma_f32+s_cmp/s_cselect/s_and")
    salu_indep = (m1 * 32 - 16 * pk) / 16 if m1 else None
    salu_dep = (m3 * 64 - 16 * pk) / 48 if m3 else None
    res = {"kernel": pmck, "waves_per_simd": waves, "valu_instructions": total,
           "valu_issue_cycles": cyc, "valu_issue_cycles_bounds": [lo, hi],
           "mean_cycles_per_valu": cyc / total,
           "salu_instructions": salu, "salu_marginal_cycles": {"independent": salu_indep, "dependent_chain": salu_dep},
           "classes": detail, "cost_source": costf, "pmc_source": pmcf, "isa_source": isa}
    json.dump(res, open(out, "w"), indent=1, sort_keys=True)
    print(json.dumps({k: res[k] for k in ("kernel", "valu_instructions", "valu_issue_cycles", "valu_issue_cycles_bounds",
                                          "mean_cycles_per_valu", "salu_instructions", "salu_marginal_cycles")}))


if __name__ == "__main__":
    main()
