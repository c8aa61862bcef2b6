"""Tuning variants of libramcrc for same-box A/B runs on the GPU box
(`python -m ramcloud_amd.build --variants [names]`, then
`RAMCRC_LIB=ramcloud_amd/lib/variants/libramcrc_<name>.so python bench.py ...`).

Kept out of build.py so that editing this bookkeeping never changes the
product library's source hash (build.source_sha covers only the sources,
headers and compile flags of the default build)."""

VARIANTS = {
    "u4_c18": ["RAMCRC_UNROLL=4", "RAMCRC_CHUNK_SHIFT=18"],
    "u2_c18": ["RAMCRC_UNROLL=2", "RAMCRC_CHUNK_SHIFT=18"],
    "u6_c18": ["RAMCRC_UNROLL=6", "RAMCRC_CHUNK_SHIFT=18"],
    "u4_c19": ["RAMCRC_UNROLL=4", "RAMCRC_CHUNK_SHIFT=19"],
    "u4_c17": ["RAMCRC_UNROLL=4", "RAMCRC_CHUNK_SHIFT=17"],
    "u4_c20": ["RAMCRC_UNROLL=4", "RAMCRC_CHUNK_SHIFT=20"],
    # parallel-walk sync search (k_walk_sync)
    "walkdbg": ["RAMCRC_WALK_DEBUG=1"],
    "fw32": ["RAMCRC_FIX_WIN_KIB=32"],
    "nocap": ["RAMCRC_NO_CAPTURE=1"],
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
    "searly": ["RAMCRC_SYNC_EARLY=1"],
    "sstrict0": ["RAMCRC_SYNC_STRICT=0"],
    "ps15": ["RAMCRC_PART_SHIFT=15"],
    "ps17": ["RAMCRC_PART_SHIFT=17"],
    "tv1": ["RAMCRC_TINY_V=1"],
    "notrim": ["RAMCRC_TINY_TRIM=0"],
    "tinyprobe": ["RAMCRC_TINY_PROBE=1", "RAMCRC_TINY_CF=0"],
    "nocf": ["RAMCRC_TINY_CF=0"],
    "bg1": ["RAMCRC_BIN_WGS_PER_CU=1"],
    "bg4": ["RAMCRC_BIN_WGS_PER_CU=4"],
    "evrec": ["RAMCRC_EXT_TIMING=0"],
    "bp2": ["RAMCRC_BIN_PER=2"],
    "bp8": ["RAMCRC_BIN_PER=8"],
    "nosafe": ["RAMCRC_TINY_SAFE=0"],
    "aa": ["RAMCRC_AA_SAME=1"],   # A/A: identical code, separate library
    # k_entries ping-pong depth / waves per CU
    "pu4": ["RAMCRC_PU=4"],
    "ew8": ["RAMCRC_ENT_WAVES=8"],
    # long-phase probes (WRONG results, A/B timing only)
    "pfold0": ["RAMCRC_PROBE_FOLD=1"],
    "pfoldcf": ["RAMCRC_PROBE_FOLD=2"],
    "pmask": ["RAMCRC_PROBE_MASK=1"],
    "pu3": ["RAMCRC_PU=3"],
    # k_entries phase stamps (tools/stamps.py)
    "stamps": ["RAMCRC_STAMPS=1"],
    "stamps_sk0": ["RAMCRC_STAMPS=1", "RAMCRC_AGE_SKEW=0"],
    "sk0": ["RAMCRC_AGE_SKEW=0"],
    "sk30": ["RAMCRC_AGE_SKEW=30"],
    "sk50": ["RAMCRC_AGE_SKEW=50"],
    "oc2": ["RAMCRC_OCTET_COST=2"],
    "sk80": ["RAMCRC_AGE_SKEW=80"],
    "ss7": ["RAMCRC_SYNC_STAGE_KIB=7"],
    "ss9": ["RAMCRC_SYNC_STAGE_KIB=9"],
    "fw8": ["RAMCRC_FIX_WIN_KIB=8"],
    "sh5_ss7": ["RAMCRC_SYNC_HOPS=5", "RAMCRC_SYNC_STAGE_KIB=7"],
    "oc6": ["RAMCRC_OCTET_COST=6"],
    "sk120": ["RAMCRC_AGE_SKEW=120"],
    "nobatch": ["RAMCRC_STEP_BATCH=0"],
}
