TAG=r02_ab_recvwt/c2 VARIANTS="base old" WL=config2 bash tools/ab.sh &&
TAG=r02_ab_recvwt/c3 VARIANTS="base old" WL=config3 bash tools/ab.sh &&
TAG=r02_ab_recvwt/c5 VARIANTS="base old send19" WL=config5 bash tools/ab.sh
