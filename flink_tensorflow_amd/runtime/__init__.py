"""L6 streaming runtime and model-aware function API."""
from .checkpoint import CheckpointStorage, RestartStrategy
from .executor import JobExecutionException, JobExecutionResult
from .functions import (AllWindowFunction, CheckpointedFunction, CoProcessFunction, Collector, FilterFunction,
                        FlatMapFunction, GlobalWindow, InitializationContext, MapFunction, OutputTag, ProcessFunction,
                        RichFlatMapFunction, RichFunction, RichMapFunction, RuntimeContext, SinkFunction,
                        SnapshotContext, SourceFunction, TimeWindow, WindowFunction)
from .model_functions import (BatchedGpuModel, CheckpointedModel, CheckpointedModelAwareFunction,
                              InputFormatModelOperations, ModelAllWindowFunction, ModelAwareFunction,
                              ModelCoProcessFunction, ModelFlatMapFunction, ModelMapFunction, ModelProcessFunction,
                              ModelWindowFunction, close_model, open_model)
from .operators import (CountWindows, SlidingEventTimeWindows, TumblingEventTimeWindows,
                        TumblingProcessingTimeWindows)
from .sources import (PROCESS_CONTINUOUSLY, PROCESS_ONCE, BytesInputFormat, CollectionSource, FileMonitoringSource,
                      FileProcessingMode, GeneratorSource, MemorySink, PrintSink, WholeFileInputFormat)
from .state import ListStateDescriptor, MapStateDescriptor, ReducingStateDescriptor, ValueStateDescriptor
from .stream import (DataStream, ExecutionConfig, KeyedStream, StreamExecutionEnvironment, register_types)

AbstractMapFunction = ModelMapFunction
AbstractFlatMapFunction = ModelFlatMapFunction
AbstractProcessFunction = ModelProcessFunction
AbstractCoProcessFunction = ModelCoProcessFunction
AbstractWindowFunction = ModelWindowFunction
AbstractAllWindowFunction = ModelAllWindowFunction
