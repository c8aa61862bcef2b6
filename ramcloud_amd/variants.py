"""Tuning variants of libramcrc for same-box A/B runs on the GPU box
(`python -m ramcloud_amd.build --variants [names]`, then
`RAMCRC_LIB=ramcloud_amd/lib/variants/libramcrc_<name>.so python bench.py ...`).

Kept out of build.py so that editing this bookkeeping never changes the
product library's source hash (build.source_sha covers only the sources,
headers and compile flags of the default build).

Every entry changes a knob away from its default and gives exact results:
tests/test_variants.py checks both (knob present in the sources, value not the
default, no knob in build.UNSAFE_DEFINES).  Libraries built from this table
report their defines in ramcrc_build_info(), and ramcrc.lib() refuses one that
names an unsafe knob."""

VARIANTS = {
    "u2": ["RAMCRC_UNROLL=2"],
    "u6": ["RAMCRC_UNROLL=6"],
    "c19": ["RAMCRC_CHUNK_SHIFT=19"],
    "c17": ["RAMCRC_CHUNK_SHIFT=17"],
    "c20": ["RAMCRC_CHUNK_SHIFT=20"],
    # parallel-walk sync search (k_walk_sync)
    "fw32": ["RAMCRC_FIX_WIN_KIB=32"],
    "ew12": ["RAMCRC_ENT_WAVES=12"],
    "sh4": ["RAMCRC_SYNC_HOPS=4"],
    "sh5": ["RAMCRC_SYNC_HOPS=5"],
    "sh3": ["RAMCRC_SYNC_HOPS=3"],
    "sh4_ss6": ["RAMCRC_SYNC_HOPS=4", "RAMCRC_SYNC_STAGE_KIB=6"],
    "sh3_ss4": ["RAMCRC_SYNC_HOPS=3", "RAMCRC_SYNC_STAGE_KIB=4"],
    "sh7": ["RAMCRC_SYNC_HOPS=7"],
    "sh8": ["RAMCRC_SYNC_HOPS=8"],
    "sh10": ["RAMCRC_SYNC_HOPS=10"],
    "sp16": ["RAMCRC_SYNC_PER=16"],
    "sp4": ["RAMCRC_SYNC_PER=4"],
    "ss6": ["RAMCRC_SYNC_STAGE_KIB=6"],
    "ss16": ["RAMCRC_SYNC_STAGE_KIB=16"],
    "ss8": ["RAMCRC_SYNC_STAGE_KIB=8"],
    "ss12": ["RAMCRC_SYNC_STAGE_KIB=12"],
    "spf0": ["RAMCRC_SYNC_PF=0"],
    "sstrict0": ["RAMCRC_SYNC_STRICT=0"],
    "ps15": ["RAMCRC_PART_SHIFT=15"],
    "ps17": ["RAMCRC_PART_SHIFT=17"],
    "notrim": ["RAMCRC_TINY_TRIM=0"],
    "nocf": ["RAMCRC_TINY_CF=0"],
    "bg1": ["RAMCRC_BIN_WGS_PER_CU=1"],
    "bg4": ["RAMCRC_BIN_WGS_PER_CU=4"],
    "evrec": ["RAMCRC_EXT_TIMING=0"],
    "bp2": ["RAMCRC_BIN_PER=2"],
    "bp8": ["RAMCRC_BIN_PER=8"],
    "nosafe": ["RAMCRC_TINY_SAFE=0"],
    # k_entries ping-pong depth / waves per CU
    "pu4": ["RAMCRC_PU=4"],
    "ew8": ["RAMCRC_ENT_WAVES=8"],
    "pu3": ["RAMCRC_PU=3"],
    # k_entries phase stamps (tools/stamps.py)
    "stamps": ["RAMCRC_STAMPS=1"],
    "stamps_sk0": ["RAMCRC_STAMPS=1", "RAMCRC_AGE_SKEW=0"],
    "sk0": ["RAMCRC_AGE_SKEW=0"],
    "sk30": ["RAMCRC_AGE_SKEW=30"],
    "sk50": ["RAMCRC_AGE_SKEW=50"],
    "oc2": ["RAMCRC_OCTET_COST=2"],
    "sk80": ["RAMCRC_AGE_SKEW=80"],
    "ss9": ["RAMCRC_SYNC_STAGE_KIB=9"],
    "fw8": ["RAMCRC_FIX_WIN_KIB=8"],
    "oc6": ["RAMCRC_OCTET_COST=6"],
    "sk120": ["RAMCRC_AGE_SKEW=120"],
    "nobatch": ["RAMCRC_STEP_BATCH=0"],
    # round 4: long-phase age skew re-tune (k_entries share per wave by age rank)
    "sk60": ["RAMCRC_AGE_SKEW=60"],
    "sk100": ["RAMCRC_AGE_SKEW=100"],
    "sk180": ["RAMCRC_AGE_SKEW=180"],
    "cu2": ["RAMCRC_COPY_U=2"],
    "cu8": ["RAMCRC_COPY_U=8"],
    "tk5": ["RAMCRC_TINY_K=5"],
    "tk6": ["RAMCRC_TINY_K=6"],
    "bo1": ["RAMCRC_BIN_ONE=1"],
    # round 5: tiny tables built in LDS from basis words (0 = copied from g_tab)
    "tg0": ["RAMCRC_TINY_GEN=0"],
    "hm0": ["RAMCRC_TINY_HM=0"],
    "pf1": ["RAMCRC_TINY_PF=1", "RAMCRC_TINY_LSEL=0"],   # round-5 start: prefetch, no selectors
    "pf0": ["RAMCRC_TINY_PF=0"],
    "md0": ["RAMCRC_TINY_MED3=0"],
    "t30": ["RAMCRC_TINY_T3=0"],
    "rg0": ["RAMCRC_TINY_REGEO=0"],
    # round 5: role split of k_entries (0: phases in sequence), kappa = tiny window cost x 1024
    "sp0": ["RAMCRC_SPLIT=0"],
    "kap128": ["RAMCRC_SPLIT_KAPPA=128"],
    "kap512": ["RAMCRC_SPLIT_KAPPA=512"],
    "kap192": ["RAMCRC_SPLIT_KAPPA=192"],
    "kap320": ["RAMCRC_SPLIT_KAPPA=320"],
    "kap224": ["RAMCRC_SPLIT_KAPPA=224"],
    "bsl1": ["RAMCRC_BIN_SLEEP=1"],
    "sy0": ["RAMCRC_SYNC_TYPES=0"],
    "m20": ["RAMCRC_TINY_M2=0"],
    "dm0": ["RAMCRC_TINY_DM=0"],
    "cnt0": ["RAMCRC_COPY_NT=0"],
    "ov0": ["RAMCRC_TINY_OVL=0"],
    "kap288": ["RAMCRC_SPLIT_KAPPA=288"],
    "bsp32": ["RAMCRC_BIN_SLEEP=32"],
    "cpf0": ["RAMCRC_COUNT_PF=0"],
    # round 6: k_walk_sync's stage always 7 KiB (the default sizes it from the mean entry)
    "sada0": ["RAMCRC_SYNC_ADAPT=0"],
    # round 6: the probe may pick 128 KiB parts again (entries of ~1.45 .. 2.9 KiB)
    "p17": ["RAMCRC_SKIP_P17=0"],
    # round 6: role split off with a heavier octet cost (the long-phase re-check)
    "sp0oc6": ["RAMCRC_SPLIT=0", "RAMCRC_OCTET_COST=6"],
}
