import cProfile, pstats, sys, os
sys.path.insert(0, os.environ.get("GRAFT_REPO_ROOT", "."))
from sfm_amd.live import KeypointStream, LiveSfM
st = KeypointStream()
frames = [st.frame(k) for k in range(300)]
s = LiveSfM(st)
for k in range(10):
    s.process(k, *frames[k][:2])
pr = cProfile.Profile()
pr.enable()
for k in range(10, 300):
    s.process(k, *frames[k][:2])
pr.disable()
ps = pstats.Stats(pr)
ps.sort_stats("cumulative")
ps.print_callees("_bundle_adjust")
print("times", s.times)
