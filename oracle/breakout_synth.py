"""TEST INFRASTRUCTURE ONLY (never imported by lightzero_amd): numpy restatement of the Breakout stand-in
game of lightzero_amd/csrc/lzm_atari.h, used to check the device env's recorded episodes.

The reference's Atari env (zoo/atari/envs/atari_lightzero_env.py) runs ALE, which is not installed: the
device env is a stand-in with Breakout's action set and frame format, so there is no reference output to
pin it to (env parity unpinned). What this file pins is the device kernel against its own specification:
`replay_episode` re-derives every frame and reward of a recorded episode from its first frame and its
actions. The one hidden random bit per serve (the ball's horizontal direction, a Philox draw on the
device) is resolved by keeping both candidates until a later frame tells them apart.
"""
import numpy as np

HW = 64
STACK = 4
BRICK_ROWS, BRICK_COLS, BRICK_Y0, BRICK_H, BRICK_W = 6, 15, 8, 2, 4
PADDLE_Y, PADDLE_W, PADDLE_SPEED = 58, 8, 3
WALL = 2
SUB = 2
AUTO_SERVE = 8
FULL_BRICKS = (1 << (BRICK_ROWS * BRICK_COLS)) - 1


def new_state(paddle):
    return dict(paddle=int(paddle), bx=0, by=0, vx=0, vy=0, in_play=0, bricks=FULL_BRICKS, lives=1, idle=0)


def render(s):
    f = np.zeros((HW, HW), np.uint8)
    f[:WALL, :] = 142
    f[:, :WALL] = 142
    f[:, HW - WALL:] = 142
    for r in range(BRICK_ROWS):
        for c in range(BRICK_COLS):
            if (s["bricks"] >> (r * BRICK_COLS + c)) & 1:
                y0, x0 = BRICK_Y0 + r * BRICK_H, WALL + c * BRICK_W
                f[y0:y0 + BRICK_H, x0:x0 + BRICK_W] = 200 - 16 * r
    f[PADDLE_Y:PADDLE_Y + 2, s["paddle"]:s["paddle"] + PADDLE_W] = 200
    if s["in_play"]:
        f[s["by"]:s["by"] + 2, s["bx"]:s["bx"] + 2] = 236
    return f


def step(s, action, serve_dir):
    """one env step (lzm_atari.h at_step); serve_dir in {+1, -1} is the serve's random direction.
    Returns (new state, raw points, terminated)."""
    s = dict(s)
    px = s["paddle"] + (PADDLE_SPEED if action == 2 else 0) - (PADDLE_SPEED if action == 3 else 0)
    px = min(max(px, WALL), HW - WALL - PADDLE_W)
    s["paddle"] = px
    if not s["in_play"]:
        s["idle"] += 1
        if action != 1 and s["idle"] < AUTO_SERVE:
            return s, 0.0, False
        s["idle"] = 0
        s.update(in_play=1, bx=px + PADDLE_W // 2 - 1, by=PADDLE_Y - 8, vx=serve_dir, vy=-1)
        return s, 0.0, False
    pts, term = 0.0, False
    x, y, vx, vy = s["bx"], s["by"], s["vx"], s["vy"]
    for _ in range(SUB):
        nx, ny = x + vx, y + vy
        if nx < WALL:
            nx, vx = WALL, -vx
        if nx > HW - WALL - 2:
            nx, vx = HW - WALL - 2, -vx
        if ny < WALL:
            ny, vy = WALL, -vy
        hit = False
        for k in range(4):
            bx, by = nx + (k & 1), ny + (k >> 1)
            if by < BRICK_Y0 or by >= BRICK_Y0 + BRICK_ROWS * BRICK_H or bx < WALL:
                continue
            r, c = (by - BRICK_Y0) // BRICK_H, (bx - WALL) // BRICK_W
            if c >= BRICK_COLS or not (s["bricks"] >> (r * BRICK_COLS + c)) & 1:
                continue
            s["bricks"] &= ~(1 << (r * BRICK_COLS + c))
            pts += 7.0 if r < 2 else (4.0 if r < 4 else 1.0)
            hit = True
            break
        if hit:
            vy, ny = -vy, y
        if vy > 0 and ny + 1 >= PADDLE_Y and ny <= PADDLE_Y + 1 and nx + 1 >= px and nx <= px + PADDLE_W - 1:
            off = (nx + 1) - (px + PADDLE_W // 2)
            vx = -2 if off < -2 else (-1 if off < 0 else (1 if off < 2 else 2))
            vy = -vy
            ny = PADDLE_Y - 2
        x, y = nx, ny
        if y > HW - 2:
            s["in_play"] = 0
            s["lives"] -= 1
            term = s["lives"] <= 0
            break
    s.update(bx=x, by=y, vx=vx, vy=vy)
    if s["bricks"] == 0:
        s["bricks"] = FULL_BRICKS
    return s, pts, term


def paddle_from_frame(frame):
    row = np.asarray(frame).reshape(HW, HW)[PADDLE_Y]
    xs = np.nonzero(row[WALL:HW - WALL] == 200)[0]
    return int(xs[0]) + WALL


def replay_episode(frames, actions, rewards, max_steps, episode_return=None):
    """frames u8 [L + 1, 64, 64] (o_0 .. o_L), actions [L], rewards [L] (clipped, as recorded), and
    optionally the recorded episode return (the unclipped score, the env's eval_episode_return).
    Re-derives the episode; returns None when it matches the game, else a message."""
    frames = np.asarray(frames).reshape(-1, HW, HW)
    L = len(actions)
    s0 = new_state(paddle_from_frame(frames[0]))
    if not np.array_equal(render(s0), frames[0]):
        return "first frame is not a reset frame"
    cands = [(s0, 0.0)]  # (game state, unclipped points so far)
    for t in range(L):
        nxt = []
        for s, score in cands:
            serve = not s["in_play"] and (int(actions[t]) == 1 or s["idle"] + 1 >= AUTO_SERVE)
            dirs = (1, -1) if serve else (1,)
            for d in dirs:
                s1, pts, term = step(s, int(actions[t]), d)
                r = 1.0 if pts > 0 else 0.0
                last = t == L - 1
                if r != float(rewards[t]) or not np.array_equal(render(s1), frames[t + 1]):
                    continue
                if term and not last:
                    continue
                if last and not (term or t + 1 >= max_steps):
                    continue
                nxt.append((s1, score + pts))
        if not nxt:
            return f"step {t}: no game state reproduces frame {t + 1} / reward {rewards[t]}"
        # identical candidates collapse
        uniq = {(tuple(sorted(c.items())), sc): (c, sc) for c, sc in nxt}
        cands = list(uniq.values())
    if episode_return is not None and not any(sc == float(episode_return) for _, sc in cands):
        return f"episode return {episode_return} is not the game's score {sorted({sc for _, sc in cands})}"
    return None
