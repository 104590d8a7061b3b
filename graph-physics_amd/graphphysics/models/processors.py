"""Drop-in EncodeProcessDecode (reference graphphysics/models/processors.py:27-137) on libmgn.

Constructor, attributes (.K, .d, .temperature, .hidden_size, .only_processor, .use_diagonal) and
state_dict keys (nodes_encoder.*, edges_encoder.*, decode_module.*, processor_list.{i}.*) match the
reference, and modules are created in the reference's order so torch.manual_seed gives the same
initial weights. forward(graph) runs encoders, the MP GraphNetBlocks and the decoder as one
autograd node on HIP kernels (gfx950); the GMM decoder heads are out of scope
(num_mixture_components must be 0).

Extra (optional) keyword: compute_dtype — torch.float32 (exact-fp32 MFMA, default) or
torch.bfloat16 (bf16 storage, fp32 accumulation); also settable via GRAPHPHYSICS_MGN_DTYPE.
"""
import torch
import torch.nn as nn

from graphphysics import _native as nat
from graphphysics.models import _engine
from graphphysics.models.layers import GraphNetBlock, build_mlp, default_compute_dtype


class EncodeProcessDecode(nn.Module):
    def __init__(self, message_passing_num: int, node_input_size: int, edge_input_size: int,
                 output_size: int, hidden_size: int = 128, only_processor: bool = False,
                 num_mixture_components: int = 0, temperature: float = None,
                 use_diagonal: bool = True, compute_dtype: torch.dtype = None):
        super().__init__()
        if num_mixture_components != 0:
            raise NotImplementedError("GMM decoder heads are outside the MI355X MGN hot path")
        self.only_processor = only_processor
        self.hidden_size = hidden_size
        self.use_diagonal = use_diagonal
        self.d = output_size
        self.K = num_mixture_components
        self.temperature = temperature
        self.message_passing_num = message_passing_num
        if not self.only_processor:
            self.nodes_encoder = build_mlp(node_input_size, hidden_size, hidden_size)
            self.edges_encoder = build_mlp(edge_input_size, hidden_size, hidden_size)
            self.decode_module = build_mlp(hidden_size, hidden_size, output_size, layer_norm=False)
        self.processor_list = nn.ModuleList(
            [GraphNetBlock(hidden_size=hidden_size) for _ in range(message_passing_num)])
        self.compute_dtype = compute_dtype or default_compute_dtype()
        self._plan = None
        _engine.flatten_parameters(self)

    # parameters live in one flat fp32 buffer; re-home them after .to()/.cuda()/.float()
    def _apply(self, fn, *args, **kwargs):
        out = super()._apply(fn, *args, **kwargs)
        _engine.flatten_parameters(self)
        self._plan = None
        for blk in self.processor_list:
            blk._plan = None
        return out

    def set_compute_dtype(self, dtype):
        self.compute_dtype = dtype
        return self

    def _get_plan(self):
        if self._plan is None:
            mlps = [] if self.only_processor else [self.nodes_encoder, self.edges_encoder,
                                                   self.decode_module]
            # encoders read the raw features (columns not padded); the decoder reads the processor's
            # (zero-padded) hidden state: one hidden-wide block, so its input gradient has the padded width
            kblocks = [] if self.only_processor else [0, 0, 1]
            for blk in self.processor_list:
                mlps += [blk.edge_block, blk.node_block]
                kblocks += [3, 2]  # [e ‖ x_i ‖ x_j], [x ‖ aggr]: hidden-wide blocks
            self._plan = _engine.ModelPlan(self, mlps, kblocks)
        return self._plan

    def forward(self, graph) -> torch.Tensor:
        x, edge_attr, edge_index = graph.x, graph.edge_attr, graph.edge_index
        nat.require_device(x)
        topo = _engine.get_topology(edge_index, x.size(0))
        plan = self._get_plan()
        return _engine.EPDFunction.apply(plan, nat.mgn_dtype(self.compute_dtype), self.only_processor,
                                         torch.is_grad_enabled(), x, edge_attr, topo, *plan.params)
