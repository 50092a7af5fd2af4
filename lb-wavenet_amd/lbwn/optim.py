"""tf.train.AdamOptimizer drop-in (train.py:178, :186) over lbwn's flat buffers."""
import torch

from . import _lib


class AdamOptimizer:
    """TF1 Adam: lr_t = lr·√(1-β2^t)/(1-β1^t); m = β1m+(1-β1)g; v = β2v+(1-β2)g²;
    θ -= lr_t·m/(√v+ε).  g = Σxent-grad/n_valid + l2_factor·θ (non-BIAS), applied by ONE
    kernel (lbwn_adam_tf1) that also advances GLOBAL_STEP / VALID_SAMPLES.  The step's plan
    status word goes with it: a step whose chain hand-off timed out is skipped on the device
    and recorded in the cumulative status (WaveNetTrain.check_status), with no host sync."""

    def __init__(self, learning_rate=0.001, beta1=0.9, beta2=0.999, epsilon=1e-8):
        self.lr, self.b1, self.b2, self.eps = float(learning_rate), float(beta1), float(beta2), float(epsilon)
        self._slots = {}

    def slots(self, net):
        key = id(net)
        if key not in self._slots:
            self._slots[key] = (torch.zeros_like(net.flat), torch.zeros_like(net.flat))
        return self._slots[key]

    def apply_gradients(self, grads_and_vars, stream=None):
        net = grads_and_vars.net
        self.apply(net, stream)

    def apply(self, net, stream=None):
        m, v = self.slots(net)
        _lib.check(net.lib.lbwn_adam_tf1(net.flat.data_ptr(), net.grad_flat.data_ptr(), m.data_ptr(), v.data_ptr(),
                                         net.layout.n_weights, net.layout.n_total, self.lr, self.b1, self.b2,
                                         self.eps, net.l2_factor, net.stats.data_ptr(), net.counters.data_ptr(),
                                         net.status_ptr(), _lib.stream_ptr(stream)))
        net.global_step_host += 1

    # ---- checkpoint state: TF's slot names (<var>/Adam = m, <var>/Adam_1 = v) ----------------
    def state_tensors(self, net):
        m, v = self.slots(net)
        out = {}
        for name, t in net.layout.views(m).items():
            out[name + '/Adam'] = t
        for name, t in net.layout.views(v).items():
            out[name + '/Adam_1'] = t
        out['Adam/step'] = net.counters[2:3]
        return out

    def load_state_tensors(self, net, loaded):
        """Restore the slots if the checkpoint has them (reference checkpoints do not:
        tmodel.py:330 saves only the model variables, so Adam restarts from zero)."""
        m, v = self.slots(net)
        with torch.no_grad():
            if 'Adam/step' not in loaded:
                m.zero_()
                v.zero_()
                net.counters[2:3].zero_()
                return False
            for name, t in net.layout.views(m).items():
                t.copy_(loaded[name + '/Adam'])
            for name, t in net.layout.views(v).items():
                t.copy_(loaded[name + '/Adam_1'])
            net.counters[2:3].copy_(loaded['Adam/step'])
        return True
