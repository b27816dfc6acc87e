"""One node of the reference's multi-process CLI over the socket broker (test helper).

usage: python tests/socket_node.py slave|master BROKER DATA.npy [K M OUT.npz] [--oracle]

--oracle (CPU tests): the node's arithmetic is the float64 oracle (oracle/ref_cpu.py,
test infrastructure) instead of the GPU path, so the transport and protocol run on
a machine without a GPU.  Without it the product nodes run (HIP kernels)."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402
import torch  # noqa: E402

from distributed_eigenspaces_amd import distributed as dd  # noqa: E402


class OracleSlave(dd.SlaveNode):
    def _device_rows(self, lo, hi):
        return torch.from_numpy(np.asarray(self.data[lo:hi], dtype=np.float64))

    def compute_sigma_hat_(self, x):
        from oracle import ref_cpu
        return torch.from_numpy(ref_cpu.sigma_hat(x.numpy()))

    def top_k_eigenvectors(self, matrix, k):
        from oracle import ref_cpu
        return torch.from_numpy(np.ascontiguousarray(ref_cpu.top_k_eigenvectors(matrix.numpy(), k)))


class OracleMaster(dd.MasterNode):
    def server_solve_(self):
        from oracle import ref_cpu
        w, v = ref_cpu.server_topk(self.computed_eigens, int(self.rank), self.batches_number)

        class R:
            pass
        r = R()
        r.evals, r.V = torch.from_numpy(w), torch.from_numpy(v)
        return r


def main():
    role, broker, path = sys.argv[1:4]
    oracle = "--oracle" in sys.argv
    data = dd.load_dataset(path)
    if role == "slave":
        node = (OracleSlave if oracle else dd.SlaveNode)(broker, data)
        node.start()  # returns when the broker closes the connection
        return
    k, m, out = int(sys.argv[4]), int(sys.argv[5]), sys.argv[6]
    master = (OracleMaster if oracle else dd.MasterNode)(broker, k, m, data)
    master.received = []
    cb = master.callback_

    def record(channel, method, properties, body):
        req = json.loads(body)
        master.received.append((req["batch"], np.array(req["eigenspace"])))
        return cb(channel, method, properties, body)
    master.channel._callbacks["master"] = record
    master.start()
    np.savez(out, ranges=np.array([r for r, _ in master.received]),
             worker_V=np.stack([v for _, v in master.received]),
             server_V=np.asarray(master.eigenspace), server_evals=np.asarray(master.eigenvalues))


if __name__ == "__main__":
    main()
