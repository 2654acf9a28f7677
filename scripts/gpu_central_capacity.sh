#!/bin/bash
# Central-topology capacity on ONE MI355X (rank 0's load at N = R + 1 GPUs, modelled with
# emulated actor links; one actor GPU's unpaced output): the table of
# profiles/r6_central_capacity.md.  Each step has its own time limit; the first failure ends it.
#   1. bench.py --actor-only E,..: one actor GPU's frames/s by envs per GPU (the capacity the
#      actor_gpu_utilisation field of the central bench divides by)
#   2. bench.py --emulate-links R --central-envs E: the learner's steps/s and the frames that
#      reach the replay, R = 1 / 3 / 7 actor links, E envs per actor GPU, one packet per link
#      per learner step
#   3. the single-GPU engine (N = 1) for the >= 95 % criterion
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/capacity
mkdir -p $O
export HSA_ENABLE_IPC_MODE_LEGACY=0
STEPS=${STEPS:-1500}
timeout -k 10 200 python bench.py --actor-only ${ACTOR_ENVS:-256,512,1024,2048} --steps 2000 --warmup 100 \
  > $O/actor_only.log 2>&1 || { echo "actor-only failed"; tail -5 $O/actor_only.log; exit 1; }
grep '^{' $O/actor_only.log | cut -c1-2000
timeout -k 10 200 python bench.py --steps $STEPS --warmup 50 > $O/n1.log 2>&1 || { echo "n1 failed"; exit 1; }
grep '^{' $O/n1.log | cut -c1-200
for E in ${CENTRAL_ENVS:-256 512 1024}; do
  for R in ${LINKS:-1 3 7}; do
    timeout -k 10 240 python bench.py --emulate-links $R --central-envs $E --steps $STEPS --warmup 50 \
      > $O/emu_R${R}_E${E}.log 2>&1 || { echo "emu R=$R E=$E failed"; tail -5 $O/emu_R${R}_E${E}.log; exit 1; }
    python - "$O/emu_R${R}_E${E}.log" "$R" "$E" <<'EOF'
import json, sys
d = json.loads([l for l in open(sys.argv[1]) if l.startswith("{")][-1])
print(json.dumps({"R": int(sys.argv[2]), "E": d["config"]["envs_per_actor_gpu"], "steps_per_s": d["value"],
                  "frames_per_s": d["actor_frames_per_sec"], "replay_ratio": d.get("replay_ratio"),
                  "actor_gpu_utilisation": d.get("actor_gpu_utilisation"),
                  "packets_per_step": d["packets_applied_per_learner_step"], "links_complete": d["links_complete"]}))
EOF
  done
done
