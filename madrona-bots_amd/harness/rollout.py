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


def learner_rollout(sim, steps, seed=1234, shift_per_species=True, fused=False, record=None, gen=None,
                    end_of_step=None):
    """The exact view pattern of learn/training_loop.py:36-137 with a learner
    stand-in instead of the models (out of scope):

        step(); species offsets (:43-45); action_tensor(False) and
        hidden_state_tensor(False) fetched ONCE (:47-48); reward / health
        clones (:49-50); per species: construct_obs(cur) (:57), its memory
        rows (:58), construct_obs(prev) (:87), PrevHiddenState rows (:89), the
        previous actions' argmax (:93); shift_observations() (:135, once per
        species -- SURVEY B.9 -- unless shift_per_species=False); then the new
        one-hot actions and memory written through the views taken before the
        shifts (:136-137).

    The stand-in's actions are torch.randint draws and its memory
    prev_memory * 0.5 + randn (both exact in float32 on any device), all drawn
    from one CPU generator, so a HIP manager and the oracle adapter given the
    same seed take the same decisions while their tables agree.  fused=True
    builds the observation rows with sim.construct_obs (one launch for all
    species) where the reference's torch.cat would read the same columns.
    `record(t, sp, name, tensor)`, when given, receives every tensor the loop
    reads (what the learner would consume), for comparison between runs;
    `end_of_step(t)` runs after each step's writes; `gen` continues the draws
    of an earlier call (a CPU torch.Generator) instead of seeding a new one."""
    if gen is None:
        gen = torch.Generator(device="cpu").manual_seed(seed)
    rec = record if record is not None else (lambda *a: None)
    agent_steps = 0
    for t in range(steps):
        sim.step()
        offsets = species_offsets(sim)
        action_tensor = sim.action_tensor(False).to_torch()
        memory_tensor = sim.hidden_state_tensor(False).to_torch()
        all_rewards = sim.reward_tensor(False).to_torch().clone()
        all_healths = sim.health_tensor(False).to_torch().clone()
        rec(t, -1, "reward", all_rewards)
        rec(t, -1, "health", all_healths)
        if fused:
            obs_all = sim.construct_obs(False)
            prev_all = sim.construct_obs(True)
        writes = []
        for sp, (s, e) in enumerate(offsets):
            if fused and not (shift_per_species and sp > 0):
                obs = obs_all[s:e]
            else:   # (after a per-species shift the fused rows are stale: rebuild)
                obs = construct_obs(sim, s, e, prev=False)
            prev_memory = memory_tensor[s:e, :]
            rec(t, sp, "obs", obs)
            rec(t, sp, "prev_memory", prev_memory)
            a = torch.randint(0, ACTION_DIM, (e - s,), generator=gen)
            noise = torch.randn((e - s, prev_memory.shape[1]), generator=gen)
            new_memory = prev_memory * 0.5 + noise.to(prev_memory.device)
            one_hot = torch.zeros(e - s, ACTION_DIM, dtype=torch.int32, device=action_tensor.device)
            one_hot.scatter_(1, a.to(action_tensor.device).unsqueeze(1), 1)
            if fused and not (shift_per_species and sp > 0):
                prev_obs = prev_all[s:e]
            else:
                prev_obs = construct_obs(sim, s, e, prev=True)
            og_hidden = sim.hidden_state_tensor(True).to_torch()[s:e, :]
            prev_actions = action_tensor[s:e, :].argmax(dim=1)
            rec(t, sp, "prev_obs", prev_obs)
            rec(t, sp, "og_hidden", og_hidden)
            rec(t, sp, "prev_actions", prev_actions)
            if shift_per_species:
                sim.shift_observations()
                action_tensor[s:e, :] = one_hot
                memory_tensor[s:e, :] = new_memory
            else:
                writes.append((s, e, one_hot, new_memory))
        if not shift_per_species:
            sim.shift_observations()
            for s, e, one_hot, new_memory in writes:
                action_tensor[s:e, :] = one_hot
                memory_tensor[s:e, :] = new_memory
        agent_steps += offsets[-1][1]
        if end_of_step is not None:
            end_of_step(t)
    return {"steps": steps, "agent_steps": agent_steps}


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
