"""L5 model abstraction and the model zoo (``models.zoo``)."""
from .core import (DefaultGraphLoader, GenericModel, GraphDefGraphLoader, GraphLoader, GraphMethod, Model,
                   ModelFunction, RichModel, default_device)
from .savedmodel import (DefaultSavedModelLoader, SavedModelBundle, SavedModelLoader, SavedModelModel,
                         SignatureConstants, TensorFlowModel, load_bundle, read_saved_model)
from .signatures import ClassificationMethod, LambdaMethod, PredictMethod, RegressionMethod
from .batched import SignatureBatchedModel

__all__ = [
    "Model", "RichModel", "GraphMethod", "ModelFunction", "GraphLoader", "DefaultGraphLoader", "GraphDefGraphLoader",
    "GenericModel", "default_device", "SignatureConstants", "SavedModelLoader", "DefaultSavedModelLoader",
    "SavedModelBundle", "TensorFlowModel", "SavedModelModel", "load_bundle", "read_saved_model", "RegressionMethod",
    "ClassificationMethod", "PredictMethod", "LambdaMethod", "SignatureBatchedModel",
]
