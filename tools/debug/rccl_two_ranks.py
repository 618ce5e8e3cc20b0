"""Probe: can two ranks share one GPU in an RCCL communicator (rt_comm_init)?"""
import os, subprocess, sys, time
sys.path[:0] = ["radiative-transfer_amd"]
if len(sys.argv) == 1:
    uidf = "/tmp/rt_uid.bin"
    if os.path.exists(uidf):
        os.remove(uidf)
    procs = [subprocess.Popen([sys.executable, __file__, str(r)]) for r in range(2)]
    rc = [p.wait(timeout=90) for p in procs]
    print("exit codes", rc)
    sys.exit(max(rc))
rank = int(sys.argv[1])
import rtsn
uidf = "/tmp/rt_uid.bin"
if rank == 0:
    open(uidf + ".tmp", "wb").write(rtsn.Comm.unique_id())
    os.rename(uidf + ".tmp", uidf)
while not os.path.exists(uidf):
    time.sleep(0.05)
uid = open(uidf, "rb").read()
try:
    c = rtsn.Comm(2, rank, uid, 0)
    print("rank", rank, "init ok", c.rank, flush=True)
    c.close()
except Exception as e:
    print("rank", rank, "init failed:", e, flush=True)
    sys.exit(3)
