"""valu_rates.py -- gfx950 VALU issue classes, the one table the issue-priority
pass (issue_prio.py) and tools/isa_report.py share.

Every VALU opcode the fast_search build may contain must be listed here, in
exactly one class; issue_prio.py exits non-zero on any other opcode, so a
compiler update that emits a new opcode stops the build instead of silently
getting a marker in the wrong place (a misplaced marker costs 4-23%,
DESIGN.md §4, profiles/r02y_kbench_marker_placement.json).

Classes (DESIGN.md §4 issue model):
  F  full rate: a wave64 instruction in 2 cycles; it can issue as the second
     instruction of a SIMD quad-cycle, beside an op of another wave.
  H  half rate or slower: 4+ cycles, never the second of a pair.

MEASURED ops were timed on MI355X by tools/valu_ops.hip
(profiles/r01d_valu_ops.json, r03b_valu_ops.json: ~115-124 lanes/clk/CU = F,
~61-63 = H, v_mov_b64 ~44, v_cndmask_b32_e32 13).  ASSUMED ops are unmeasured;
all but the per-nonce loop's one compare occur only outside that loop (digit
formatting, the candidate scan, the wave/workgroup reduction).  They are
classed by their nearest measured sibling: compares with v_cmp_lt_u32_e32
(H), 64-bit ops, lane reads/writes and mbcnt -> H.  The rate belongs to the
opcode, and not by any rule one could guess: v_lshrrev_b32 is full rate in
both encodings, v_lshlrev_b32 half in both; v_add_u32_e64 is full rate,
v_cndmask_b32 half in both.
"""

FULL_MEASURED = frozenset({
    "v_add_u32_e32", "v_add_u32_e64", "v_sub_u32_e32", "v_sub_u32_e64", "v_xor_b32_e32", "v_and_b32_e32",
    "v_or_b32_e32", "v_not_b32_e32", "v_bitop3_b32", "v_lshrrev_b32_e32", "v_lshrrev_b32_e64",
    "v_mov_b32_e32", "v_fma_f32", "v_mul_f32_e32",
})
HALF_MEASURED = frozenset({
    "v_alignbit_b32", "v_alignbyte_b32", "v_add3_u32", "v_xad_u32", "v_bfi_b32", "v_lshl_or_b32",
    "v_lshl_add_u32", "v_and_or_b32", "v_or3_b32", "v_perm_b32", "v_cndmask_b32_e64", "v_mad_u32_u24",
    "v_lshrrev_b64", "v_mov_b64", "v_mov_b64_e32", "v_lshlrev_b32_e64", "v_pk_add_u16", "v_pk_add_f32",
    "v_pk_mov_b32", "v_xor_b32_sdwa",
    # round 3 (profiles/r03b_valu_ops.json): note v_lshlrev_b32_e32 is half rate, v_lshrrev_b32 full
    "v_lshlrev_b32_e32", "v_min_u32_e32", "v_min3_u32", "v_min_u32_dpp", "v_mov_b32_dpp",
    "v_cndmask_b32_e32", "v_cmp_lt_u32_e32", "v_mul_lo_u32", "v_mul_hi_u32", "v_add_lshl_u32",
})
FULL_ASSUMED = frozenset({
    "v_subrev_u32_e32",
})
HALF_ASSUMED = frozenset({
    "v_lshlrev_b64", "v_lshl_add_u64", "v_mad_u64_u32", "v_readlane_b32", "v_writelane_b32",
    "v_readfirstlane_b32", "v_mbcnt_lo_u32_b32", "v_mbcnt_hi_u32_b32",
    # compares: their measured sibling v_cmp_lt_u32_e32 issues at half rate; the per-nonce loop's
    # v_cmp_ge_u32_e32 (h0 <= the wave's best) is classed with it (A/B: profiles/r03c_*, cmpH)
    "v_cmp_eq_u32_e32", "v_cmp_ne_u32_e32", "v_cmp_le_u32_e32", "v_cmp_gt_u32_e32", "v_cmp_ge_u32_e32",
    "v_cmp_eq_u32_e64", "v_cmp_ne_u32_e64", "v_cmp_lt_u32_e64", "v_cmp_le_u32_e64",
    "v_cmp_gt_u32_e64", "v_cmp_ge_u32_e64",
    "v_cmp_eq_u64_e32", "v_cmp_ne_u64_e32", "v_cmp_lt_u64_e32", "v_cmp_le_u64_e32",
    "v_cmp_gt_u64_e32", "v_cmp_ge_u64_e32",
    "v_cmp_eq_u64_e64", "v_cmp_ne_u64_e64", "v_cmp_lt_u64_e64", "v_cmp_le_u64_e64",
    "v_cmp_gt_u64_e64", "v_cmp_ge_u64_e64",
})
FULL = FULL_MEASURED | FULL_ASSUMED
HALF = HALF_MEASURED | HALF_ASSUMED
assert not (FULL & HALF)


class UnknownOpcode(ValueError):
    pass


def valu_rate(op):
    """'F' or 'H' for a VALU mnemonic as printed by the gfx950 assembler
    (encoding suffix included); UnknownOpcode for anything unlisted."""
    if op in FULL:
        return "F"
    if op in HALF:
        return "H"
    raise UnknownOpcode(f"VALU opcode {op!r} has no issue class in valu_rates.py: measure it "
                        "(tools/valu_ops.hip) and add it to FULL_* or HALF_*")
