"""TEST INFRASTRUCTURE ONLY (never imported by lightzero_amd): numpy restatement of the Pong stand-in game of
lightzero_amd/csrc/lzm_atari.h (GAME = 1, pg_*), used to check the device env's recorded episodes.

The reference's Atari env (zoo/atari/envs/atari_lightzero_env.py) runs ALE, which is not installed: the device
env is a stand-in with Pong's action set and frame format, so there is no reference output to pin it to (env
parity unpinned). What this file pins is the device kernel against its own specification: `replay_episode`
re-derives every frame and reward of a recorded episode from its first frame and its actions. The two hidden
random bits per serve (the ball's directions, a Philox draw on the device) are resolved by keeping every
candidate until a later frame tells them apart.
"""
import numpy as np

HW = 64
WALL = 2
SUB = 2
PADDLE_H, SPEED, OPP_SPEED, ME_X, OPP_X, AUTO_SERVE, WIN = 8, 3, 2, 56, 6, 8, 21
COURT, WALL_V, ME_V, OPP_V, BALL_V = 87, 236, 147, 130, 236


def new_state(paddle, opp):
    return dict(paddle=int(paddle), opp=int(opp), bx=0, by=0, vx=0, vy=0, in_play=0, me=0, them=0, idle=0)


def clamp_paddle(y):
    return min(max(y, WALL), HW - WALL - PADDLE_H)


def bounce_vy(off):
    return -2 if off < -2 else (-1 if off < 0 else (1 if off < 2 else 2))


def render(s):
    f = np.full((HW, HW), COURT, np.uint8)
    f[:WALL, :] = WALL_V
    f[HW - WALL:, :] = WALL_V
    f[s["paddle"]:s["paddle"] + PADDLE_H, ME_X:ME_X + 2] = ME_V
    f[s["opp"]:s["opp"] + PADDLE_H, OPP_X:OPP_X + 2] = OPP_V
    if s["in_play"]:
        f[s["by"]:s["by"] + 2, s["bx"]:s["bx"] + 2] = BALL_V
    return f


def step(s, action, serve_bits):
    """one env step (lzm_atari.h pg_step); serve_bits (0..3) the serve's random draw. Returns (state, points,
    terminated)."""
    s = dict(s)
    up, down = action in (2, 4), action in (3, 5)
    fire = action in (1, 4, 5)
    py = clamp_paddle(s["paddle"] + (-SPEED if up else 0) + (SPEED if down else 0))
    s["paddle"] = py
    if not s["in_play"]:
        s["idle"] += 1
        if not fire and s["idle"] < AUTO_SERVE:
            return s, 0.0, False
        s["idle"] = 0
        s.update(in_play=1, bx=HW // 2 - 1, by=HW // 2 - 1, vx=1 if serve_bits & 1 else -1,
                 vy=1 if serve_bits & 2 else -1)
        return s, 0.0, False
    pts, term = 0.0, False
    x, y, vx, vy, oy = s["bx"], s["by"], s["vx"], s["vy"], s["opp"]
    for _ in range(SUB):
        oc, bc = oy + PADDLE_H // 2, y + 1
        oy = clamp_paddle(oy + (OPP_SPEED if bc > oc + 1 else (-OPP_SPEED if bc < oc - 1 else 0)))
        nx, ny = x + vx, y + vy
        if ny < WALL:
            ny, vy = WALL, -vy
        if ny > HW - WALL - 2:
            ny, vy = HW - WALL - 2, -vy
        if vx > 0 and nx + 1 >= ME_X and nx <= ME_X + 1 and ny + 1 >= py and ny <= py + PADDLE_H - 1:
            vy, vx, nx = bounce_vy((ny + 1) - (py + PADDLE_H // 2)), -vx, ME_X - 2
        elif vx < 0 and nx <= OPP_X + 1 and nx + 1 >= OPP_X and ny + 1 >= oy and ny <= oy + PADDLE_H - 1:
            vy, vx, nx = bounce_vy((ny + 1) - (oy + PADDLE_H // 2)), -vx, OPP_X + 2
        x, y = nx, ny
        if x < 0 or x > HW - 2:
            mine = x < 0
            pts = 1.0 if mine else -1.0
            s["me" if mine else "them"] += 1
            s["in_play"] = 0
            term = s["me"] >= WIN or s["them"] >= WIN
            break
    s.update(bx=x, by=y, vx=vx, vy=vy, opp=oy)
    return s, pts, term


def paddles_from_frame(frame):
    f = np.asarray(frame).reshape(HW, HW)
    me = np.nonzero(f[:, ME_X] == ME_V)[0]
    opp = np.nonzero(f[:, OPP_X] == OPP_V)[0]
    return int(me[0]), int(opp[0])


def replay_episode(frames, actions, rewards, max_steps, episode_return=None):
    """frames u8 [L + 1, 64, 64] (o_0 .. o_L), actions [L], rewards [L] (clipped, as recorded), and optionally
    the recorded episode return (the point difference, the env's eval_episode_return). Re-derives the episode;
    returns None when it matches the game, else a message."""
    frames = np.asarray(frames).reshape(-1, HW, HW)
    L = len(actions)
    s0 = new_state(*paddles_from_frame(frames[0]))
    if not np.array_equal(render(s0), frames[0]):
        return "first frame is not a reset frame"
    cands = [(s0, 0.0)]
    for t in range(L):
        nxt = []
        for s, score in cands:
            serve = not s["in_play"] and (int(actions[t]) in (1, 4, 5) or s["idle"] + 1 >= AUTO_SERVE)
            for bits in ((0, 1, 2, 3) if serve else (0,)):
                s1, pts, term = step(s, int(actions[t]), bits)
                last = t == L - 1
                if float(np.sign(pts)) != float(rewards[t]) or not np.array_equal(render(s1), frames[t + 1]):
                    continue
                if term and not last:
                    continue
                if last and not (term or t + 1 >= max_steps):
                    continue
                nxt.append((s1, score + pts))
        if not nxt:
            return f"step {t}: no game state reproduces frame {t + 1} / reward {rewards[t]}"
        uniq = {(tuple(sorted(c.items())), sc): (c, sc) for c, sc in nxt}
        cands = list(uniq.values())
    if episode_return is not None and not any(sc == float(episode_return) for _, sc in cands):
        return f"episode return {episode_return} is not the game's score {sorted({sc for _, sc in cands})}"
    return None
