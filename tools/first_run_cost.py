import sys, time
sys.path.insert(0, "/root/repo/cop5615-gossip_protocol_amd")
from gossip_amd import Simulator
for n, t, a in [(1000, "full", "gossip"), (100000, "3D", "push-sum"), (1000, "line", "push-sum")]:
    s = Simulator(n, t, a, seed=1)
    for i in range(3):
        s.reset()
        st = s.step(1 << 40)
        print(n, t, a, "run", i, "rounds", st.round, "device_ms %.3f" % st.device_ms, flush=True)
    s.close()
