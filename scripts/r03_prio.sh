#!/bin/bash
# Round 3 wave-priority measurements on one box: step-kernel A/B (solver phase at priority 1 vs 0),
# the policy kernels with a static priority for one half of the waves, the -m gpu suite, smoke and
# the default bench line, the CG solver line, then the actor-in-the-loop legs with the slot-sized
# actor at priority 2 (a variant library copied over the product one, last). Usage: <tag>
set -e -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
T=$1
O=gpurun_out/$T
mkdir -p $O
ROUNDS=9 bash scripts/r03_ab3.sh $T evariants/libeng_base2.so evariants/libeng_prio0.so evariants/libeng_prio.so
timeout -k 10 300 python3 scripts/policy_variants.py run > $O/pol_actor.log 2>&1
ZB_POL_KIND=critic timeout -k 10 300 python3 scripts/policy_variants.py run > $O/pol_critic.log 2>&1
bash scripts/r03_check.sh $T
L="--no-cpu-baseline --no-ppo --no-policy --no-pipeline --no-c2-rollout"
timeout -k 10 300 python3 bench.py --solver cg $L > $O/bench_cg.json 2> $O/bench_cg.err
P="--no-cpu-baseline --no-ppo --no-c2-rollout"
timeout -k 10 300 python3 bench.py $P > $O/bench_pol_base.json 2> $O/bench_pol_base.err
cp variants/libzbot_polprio2.so ksim-gym-zbot_amd/zbot_amd/libzbot_hip.so
timeout -k 10 300 python3 bench.py $P > $O/bench_pol_prio2.json 2> $O/bench_pol_prio2.err
