"""Hot-path-relevant defaults of arguments/__init__.py:50-125 (ModelParams / PipelineParams /
OptimizationParams) as plain objects; `is_blender` is a real true/false flag here."""


class ModelParams:
    def __init__(self, **kw):
        self.sh_degree = 3
        self.white_background = False
        self.is_blender = True
        self.is_6dof = False
        self.D, self.W, self.multires = 8, 256, 10
        self.__dict__.update(kw)


class PipelineParams:
    def __init__(self, **kw):
        self.convert_SHs_python = False
        self.compute_cov3D_python = False
        self.debug = False
        self.__dict__.update(kw)


class OptimizationParams:
    def __init__(self, **kw):
        self.iterations = 40_000
        self.warm_up = 3000
        self.position_lr_init = 0.00016
        self.position_lr_final = 0.0000016
        self.position_lr_delay_mult = 0.01
        self.position_lr_max_steps = 30_000
        self.deform_lr_max_steps = 40_000
        self.feature_lr = 0.0025
        self.opacity_lr = 0.05
        self.scaling_lr = 0.001
        self.rotation_lr = 0.001
        self.percent_dense = 0.01
        self.lambda_dssim = 0.2
        self.densification_interval = 100
        self.opacity_reset_interval = 3000
        self.densify_from_iter = 500
        self.densify_until_iter = 15_000
        self.densify_grad_threshold = 0.0007
        self.sequence_length = 30
        self.__dict__.update(kw)
