"""EC16P20L2 fused encode through the ec seam (dev check, round 4): which kernel the library takes for
the LRC code mode's 22 rows (20 global + 2 AZ-local parities) and its time per call, for A/B with
CFSEC_BS16=0 under rocprofv3 --kernel-trace --stats.  64 bids x S = 262,144 in HBM, three tasklets
in rotation; the parity of tasklet 0 is checksummed (sha256) so two runs can be compared."""
import hashlib
import sys
import time

import torch

sys.path.insert(0, ".")
from chubaofs_amd import codemode as cm, ec  # noqa: E402

t5 = cm.GetTactic(cm.EC16P20L2)
n, nb, S = t5.N + t5.M + t5.L, 64, 262144
dev = torch.device("cuda", 0)
enc = ec.NewEncoder(ec.Config(CodeMode=t5, EnableVerify=False), device=0)
g = torch.Generator(device=dev)
g.manual_seed(0xC5)
tasks = []
for _ in range(3):
    full = torch.zeros((nb, n, S), dtype=torch.uint8, device=dev)
    full[:, :t5.N] = torch.randint(0, 256, (nb, t5.N, S), generator=g, device=dev, dtype=torch.uint8)
    tasks.append((full, [[full[b, i] for i in range(n)] for b in range(nb)]))
for i in range(6):
    assert enc.EncodeBatchAsync(tasks[i % 3][1]) == [0] * nb
torch.cuda.synchronize()
reps = 30
t0 = time.perf_counter()
for i in range(reps):
    enc.EncodeBatchAsync(tasks[i % 3][1])
torch.cuda.synchronize()
dt = (time.perf_counter() - t0) / reps
print(f"EC16P20L2 encode_batch_async, 64 x 262144: {dt * 1e6:.1f} us per call (wall, back to back)")
print("parity sha256 of tasklet 0:", hashlib.sha256(tasks[0][0][:, t5.N:].cpu().numpy().tobytes()).hexdigest()[:32])
