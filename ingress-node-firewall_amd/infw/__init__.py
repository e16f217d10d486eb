"""infw — MI355X-native batched ingress-firewall classifier (host side).

Package layout (ingress-node-firewall_amd/):
  csrc/     HIP kernels (classify.hip), table compiler, C ABI (include/infw.h)
  lib/      libinfw.so (product) and libinfw_workload.so (bench/test workloads), built in-tree
  infw/     this Python mirror of the reference's pkg/ebpf + pkg/metrics API over the C ABI
"""
from ._native import (build_id, BPF_ANY, BPF_EXIST, BPF_NOEXIST, COMMIT_FULL, COMMIT_INCREMENTAL, COMMIT_REUPLOAD,
                      F_FULL_COMMIT, F_HOST_ONLY, F_KEEP_HOST_IMAGE, LIB_PATH, MAX_TARGETS,
                      INPUT_COMPACT, INPUT_FRAMES, INPUT_SOA, INPUT_XDP, XDP_DROP, XDP_PASS, InfwError, LpmIpKeySt,
                      RuleStatisticsSt, RulesValSt, RuleTypeSt, kernel_variants, option_names)
from .core import (DEFAULT_OPTIONS, Classifier, HostSoa, build_ebpf_key, compact_to_tuples, key_from_fields,
                   pack_xdp_host, verdicts_from_results, xdp_host_events, Burst, BurstArray, pack_burst_host,
                   burst_host_events)
from .controller import (IngNodeFwController, IngressNodeFirewallRules, ProtocolRule, Statistics,
                         make_rules_val)

__all__ = [
    "Classifier", "HostSoa", "pack_xdp_host", "xdp_host_events", "Burst", "BurstArray", "pack_burst_host", "burst_host_events", "compact_to_tuples", "build_ebpf_key", "key_from_fields", "verdicts_from_results", "IngNodeFwController",
    "IngressNodeFirewallRules", "ProtocolRule", "Statistics", "make_rules_val", "LpmIpKeySt", "RulesValSt",
    "RuleTypeSt", "RuleStatisticsSt", "InfwError", "BPF_ANY", "BPF_NOEXIST", "BPF_EXIST", "F_HOST_ONLY",
    "build_id", "DEFAULT_OPTIONS", "INPUT_SOA", "INPUT_COMPACT", "INPUT_FRAMES", "INPUT_XDP", "kernel_variants", "option_names",
    "F_KEEP_HOST_IMAGE", "F_FULL_COMMIT", "COMMIT_FULL", "COMMIT_INCREMENTAL", "COMMIT_REUPLOAD", "XDP_DROP", "XDP_PASS", "MAX_TARGETS", "LIB_PATH",
]
