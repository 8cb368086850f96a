"""Static / dynamic loss scaling (reference `runtime/fp16/loss_scaler.py:91-270`, same update rule: halve on
overflow after `delayed_shift` hysteresis, double after `scale_window` clean steps, floor at `min_scale`)."""
import torch

INITIAL_LOSS_SCALE = "init_scale"
SCALE_WINDOW = "scale_window"
DELAYED_SHIFT = "delayed_shift"
CONSECUTIVE_HYSTERESIS = "consecutive_hysteresis"
MIN_LOSS_SCALE = "min_scale"


class LossScalerBase:

    def __init__(self, cur_scale):
        self.cur_scale = cur_scale
        self.dynamic = False

    @property
    def loss_scale(self):
        return self.cur_scale

    def scale_gradient(self, module, grad_in, grad_out):
        return tuple(self.loss_scale * g for g in grad_in)

    def update_scale(self, overflow):
        pass

    def backward(self, loss, retain_graph=False):
        (loss * self.loss_scale).backward(retain_graph=retain_graph)

    # plain-dict state so checkpoints stay loadable with torch.load(weights_only=True)
    def state_dict(self):
        d = {k: (str(v) if isinstance(v, torch.dtype) else v) for k, v in vars(self).items()}
        d["type"] = type(self).__name__
        return d

    def load_state_dict(self, d):
        for k, v in d.items():
            if k == "type":
                continue
            if k == "dtype" and isinstance(v, str):
                v = getattr(torch, v.replace("torch.", ""))
            setattr(self, k, v)


class LossScaler(LossScalerBase):

    def __init__(self, scale=1):
        super().__init__(scale)

    def has_overflow(self, params):
        return False


class DynamicLossScaler(LossScalerBase):

    def __init__(self, init_scale=2**32, scale_factor=2.0, scale_window=1000, min_scale=1, delayed_shift=1,
                 consecutive_hysteresis=False, raise_error_at_min_scale=True, dtype=torch.half):
        super().__init__(init_scale)
        self.cur_iter = 0
        self.last_overflow_iter = -1
        self.scale_factor = scale_factor
        self.scale_window = scale_window
        self.min_scale = min_scale
        self.delayed_shift = delayed_shift
        self.cur_hysteresis = delayed_shift
        self.consecutive_hysteresis = consecutive_hysteresis
        self.raise_error_at_min_scale = raise_error_at_min_scale
        self.dynamic = True
        self.dtype = dtype

    def _shrink(self):
        if self.cur_scale == self.min_scale and self.raise_error_at_min_scale:
            raise Exception("Current loss scale already at minimum - cannot decrease scale anymore. Exiting run.")
        self.cur_scale = max(self.cur_scale / self.scale_factor, self.min_scale)

    def update_scale(self, overflow):
        """One optimizer step's verdict. An overflow first spends the hysteresis budget (`delayed_shift` - 1 free
        passes), then divides the scale; `scale_window` steps since the last overflow multiply it back. The budget
        refills on every clean step (`consecutive_hysteresis`) or only when the scale grows."""
        step = self.cur_iter
        self.cur_iter = step + 1
        if overflow:
            self.last_overflow_iter = step
            if self.delayed_shift > 1 and self.cur_hysteresis > 1:
                self.cur_hysteresis -= 1
            else:
                self._shrink()
            return
        if self.consecutive_hysteresis:
            self.cur_hysteresis = self.delayed_shift
        if (step - self.last_overflow_iter) % self.scale_window == 0:
            if not self.consecutive_hysteresis:
                self.cur_hysteresis = self.delayed_shift
            self.cur_scale *= self.scale_factor


def CreateLossScaler(dtype, static_loss_scale, dynamic_scaling, dynamic_loss_args):
    if dtype == torch.half and dynamic_scaling:
        if dynamic_loss_args is None:
            return DynamicLossScaler(dtype=dtype)
        return DynamicLossScaler(dtype=dtype, **dynamic_loss_args)
    return LossScaler(scale=static_loss_scale if dtype == torch.half else 1.0)
