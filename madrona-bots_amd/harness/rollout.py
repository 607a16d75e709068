"""Rollout harness -- the call sequence of learn/env.py:44-104 and
learn/training_loop.py:29-137 without the learner math (out of scope):

    step() -> species offsets (species_count_tensor().sum(0).cumsum(0),
    env.py:55-57) -> per species construct_obs(cur) / construct_obs(prev)
    (learn/util.py:14-29) -> sample actions -> shift_observations() ->
    write one-hot actions into action_tensor rows (env.py:94-98).

Works with anything exposing the SimManager surface: madrona_bots.SimManager
with exec_mode "hip" (a GPU) or "cpu" (BASELINE config 1: 64 worlds without a
GPU; like learn/env.py:12-15 the default picks cpu when no GPU is present).

    python madrona-bots_amd/harness/rollout.py --worlds 4096 --steps 100
    python madrona-bots_amd/harness/rollout.py --worlds 64 --exec-mode cpu
"""
import argparse
import json
import os
import sys
import time

import torch

NUM_SPECIES = 4
OBS_DIM = 69        # depth 32 + health 1 + position 2 + semantic 32 + surrounding 2 (env.py:19)
ACTION_DIM = 6


def species_offsets(sim):
    """learn/env.py:55-57: [start, end) export rows of each species."""
    counts = sim.species_count_tensor().to_torch()
    end = counts.sum(dim=0).cumsum(dim=0)
    start = torch.cat((torch.zeros(1, dtype=end.dtype, device=end.device), end[:-1]))
    return [(int(s), int(e)) for s, e in zip(start.tolist(), end.tolist())]


def construct_obs(sim, start, end, prev=False):
    """learn/util.py:14-29 (torch.cat promotes the uint8/int8/f32 pieces to f32)."""
    return torch.cat((sim.depth_tensor(prev).to_torch()[start:end, :],
                      sim.health_tensor(prev).to_torch()[start:end, :],
                      sim.position_tensor(prev).to_torch()[start:end, :],
                      sim.semantic_tensor(prev).to_torch()[start:end, :],
                      sim.surrounding_tensor(prev).to_torch()[start:end, :]), dim=1)


def random_rollout(sim, steps, seed=1234, shift_per_species=False, device=None, fused=False):
    """Random-action rollout (BASELINE config 2).  shift_per_species=True
    reproduces the reference's shift inside the species loop.
    fused=True builds the observation rows with sim.construct_obs (one kernel
    for all species, sliced per species) instead of the 5-way torch.cat."""
    gen = torch.Generator(device=device if device is not None else "cpu").manual_seed(seed)
    stats = {"steps": 0, "agent_steps": 0, "step_s": 0.0, "obs_rows": 0}
    for t in range(steps):
        t0 = time.perf_counter()
        sim.step()
        if device is not None and device.type == "cuda":
            torch.cuda.synchronize(device)
        stats["step_s"] += time.perf_counter() - t0
        offsets = species_offsets(sim)
        action = sim.action_tensor(False).to_torch()
        new_actions = []
        if fused:
            # the previous rows first: they need no sensor rows, so their
            # kernel runs beside the sensor instead of queueing behind the
            # current rows' wait for it (the two reads are independent)
            prev_all = sim.construct_obs(True) if t > 0 else None
            obs_all = sim.construct_obs(False)
        for sp, (s, e) in enumerate(offsets):
            if fused and not (shift_per_species and sp > 0):
                obs = obs_all[s:e]
                prev = prev_all[s:e] if prev_all is not None else None
            else:   # after a per-species shift the prev rows changed: rebuild
                obs = construct_obs(sim, s, e, prev=False)
                prev = construct_obs(sim, s, e, prev=True) if t > 0 else None
            assert obs.shape == (e - s, OBS_DIM) and obs.dtype == torch.float32
            if prev is not None:
                assert prev.shape == obs.shape
            stats["obs_rows"] += e - s
            a = torch.randint(0, ACTION_DIM, (e - s,), generator=gen, device=gen.device)
            one_hot = torch.zeros(e - s, ACTION_DIM, dtype=torch.int32, device=action.device)
            one_hot.scatter_(1, a.to(action.device).unsqueeze(1), 1)
            new_actions.append((s, e, one_hot))
            if shift_per_species:
                sim.shift_observations()
                action[s:e, :] = one_hot
        if not shift_per_species:
            sim.shift_observations()
            for s, e, one_hot in new_actions:
                action[s:e, :] = one_hot
        stats["steps"] += 1
        stats["agent_steps"] += offsets[-1][1]
    return stats


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--worlds", type=int, default=4096)
    ap.add_argument("--steps", type=int, default=100)
    ap.add_argument("--seed", type=int, default=69)
    ap.add_argument("--agents", type=int, default=32)
    ap.add_argument("--fused", action="store_true", help="sim.construct_obs instead of torch.cat")
    ap.add_argument("--exec-mode", default="auto", choices=("auto", "hip", "cpu"),
                    help="auto: hip when a GPU is present, else cpu (learn/env.py:12-15)")
    a = ap.parse_args()
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    import madrona_bots as mb
    mode = a.exec_mode if a.exec_mode != "auto" else ("hip" if torch.cuda.is_available() else "cpu")
    dev = torch.device("cuda", 0) if mode == "hip" else torch.device("cpu")
    sim = mb.SimManager(0, a.worlds, a.seed, a.agents, exec_mode=mode)
    random_rollout(sim, 5, device=dev, fused=a.fused)
    st = random_rollout(sim, a.steps, device=dev, fused=a.fused)
    # the reference's "Average FPS for simulator" = num_worlds / mean step time
    print(json.dumps({"worlds": a.worlds, "exec_mode": mode, "steps": st["steps"],
                      "world_steps_per_s": a.worlds * st["steps"] / st["step_s"],
                      "agent_steps_per_s_step_only": st["agent_steps"] / st["step_s"]}))


if __name__ == "__main__":
    main()
