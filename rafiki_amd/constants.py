"""String enums shared by every layer (wire values identical to reference rafiki/constants.py:1-62)."""


class BudgetType:
    MODEL_TRIAL_COUNT = 'MODEL_TRIAL_COUNT'
    GPU_COUNT = 'GPU_COUNT'
    TIME_HOURS = 'TIME_HOURS'  # extension: wall-clock budget per sub-train-job


class ModelDependency:
    TENSORFLOW = 'tensorflow'
    KERAS = 'Keras'
    SCIKIT_LEARN = 'scikit-learn'
    PYTORCH = 'torch'
    SINGA = 'singa'


class ModelAccessRight:
    PUBLIC = 'PUBLIC'
    PRIVATE = 'PRIVATE'


class InferenceJobStatus:
    STARTED = 'STARTED'
    RUNNING = 'RUNNING'
    ERRORED = 'ERRORED'
    STOPPED = 'STOPPED'


class TrainJobStatus:
    STARTED = 'STARTED'
    RUNNING = 'RUNNING'
    STOPPED = 'STOPPED'
    ERRORED = 'ERRORED'


class TrialStatus:
    STARTED = 'STARTED'
    RUNNING = 'RUNNING'
    ERRORED = 'ERRORED'
    TERMINATED = 'TERMINATED'
    COMPLETED = 'COMPLETED'


class ServiceStatus:
    STARTED = 'STARTED'
    DEPLOYING = 'DEPLOYING'
    RUNNING = 'RUNNING'
    ERRORED = 'ERRORED'
    STOPPED = 'STOPPED'


class ServiceType:
    TRAIN = 'TRAIN'
    PREDICT = 'PREDICT'
    INFERENCE = 'INFERENCE'


class UserType:
    SUPERADMIN = 'SUPERADMIN'
    ADMIN = 'ADMIN'
    MODEL_DEVELOPER = 'MODEL_DEVELOPER'
    APP_DEVELOPER = 'APP_DEVELOPER'


class AdvisorType:
    BTB_GP = 'BTB_GP'        # reference name; served by our GP-EI Bayesian optimiser
    GP_EI = 'GP_EI'
    RANDOM = 'RANDOM'


class DatasetType:
    IMAGE_FILES = 'IMAGE_FILES'
    CORPUS = 'CORPUS'


class TaskType:
    IMAGE_CLASSIFICATION = 'IMAGE_CLASSIFICATION'
    POS_TAGGING = 'POS_TAGGING'
    IMAGE_GENERATION = 'IMAGE_GENERATION'
