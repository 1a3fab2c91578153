#!/bin/bash
# Send direction write-through stores at 4 workgroups per CU (n1: WS
# serialize; n2: and the fused HTTP/2 send; n3: n2 with sc1 nt) against the
# current build, configs 2, 3 and 5.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
TAG=r02_ab_sendwt/c2 VARIANTS="base n1 n3" WL=config2 bash tools/ab.sh &&
TAG=r02_ab_sendwt/c3 VARIANTS="base n1" WL=config3 bash tools/ab.sh &&
TAG=r02_ab_sendwt/c5 VARIANTS="base n1 n2 n3" WL=config5 bash tools/ab.sh
