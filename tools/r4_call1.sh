#!/bin/bash
# dist checks, then the gemm_xs waves A/B (stops on a timeout / crash exit of either)
bash tools/r4_dist.sh; rc=$?
case $rc in 124|134|137|139) exit $rc;; esac
bash tools/r4_xs_ab.sh
