"""Where the live path's host time goes: bench.py's live_path_leg loop (300
synthetic frames, same warm-up) under cProfile; prints the phase totals and
the functions with the largest cumulative time, with call counts.
  python tools/live_profile.py [n_frames] [top]"""
import cProfile
import os
import pstats
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from sfm_amd.live import KeypointStream, LiveSfM  # noqa: E402


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 300
    top = int(sys.argv[2]) if len(sys.argv) > 2 else 45
    st = KeypointStream()
    frames = [st.frame(k)[:2] for k in range(n)]
    warm = LiveSfM(st)
    for k in range(25):
        warm.process(k, *frames[k])
    warm.close()
    s = LiveSfM(st)
    t0 = time.perf_counter()
    for k in range(n):
        s.process(k, *frames[k])
    plain = time.perf_counter() - t0
    s.close()
    s = LiveSfM(st)
    pr = cProfile.Profile()
    pr.enable()
    for k in range(n):
        s.process(k, *frames[k])
    pr.disable()
    print(f"unprofiled {plain / n * 1e3:.3f} ms/frame; phases (profiled run) "
          f"{ {k: round(v, 4) for k, v in s.times.items()} }", flush=True)
    s.close()
    pstats.Stats(pr).sort_stats("cumulative").print_stats(top)
    pstats.Stats(pr).sort_stats("tottime").print_stats(25)


if __name__ == "__main__":
    main()
