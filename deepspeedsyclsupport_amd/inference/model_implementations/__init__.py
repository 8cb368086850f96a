from .transformer import DSInferenceLayer, DSInferenceModel, DSModelSpec
