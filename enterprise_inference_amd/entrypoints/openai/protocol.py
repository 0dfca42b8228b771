"""OpenAI-compatible request/response schemas.

Field lists follow the reference's published contract, docs/api-spec.yaml:
ChatCompletionRequest (:259, 45 fields incl. the vLLM extras ``top_k``, ``min_p``,
``repetition_penalty``, ``guided_*``, ``chat_template_kwargs``), CompletionRequest
(:614, 40 fields), EmbeddingRequest (:880).  Unknown fields are accepted and
ignored, like vLLM's server.
"""

from __future__ import annotations

import time
import uuid
from typing import Any, Dict, List, Literal, Optional, Union

from pydantic import BaseModel, ConfigDict, Field

from ...engine.sampling_params import SamplingParams


def random_id(prefix: str) -> str:
    return f"{prefix}-{uuid.uuid4().hex}"


class OpenAIBase(BaseModel):
    model_config = ConfigDict(extra="allow", protected_namespaces=())


class ErrorResponse(OpenAIBase):
    object: str = "error"
    message: str
    type: str
    param: Optional[str] = None
    code: int


class StreamOptions(OpenAIBase):
    include_usage: Optional[bool] = False
    continuous_usage_stats: Optional[bool] = False


class ResponseFormat(OpenAIBase):
    type: Literal["text", "json_object", "json_schema"] = "text"
    json_schema: Optional[Dict[str, Any]] = None


class FunctionDefinition(OpenAIBase):
    name: str
    description: Optional[str] = None
    parameters: Optional[Dict[str, Any]] = None


class ChatCompletionToolsParam(OpenAIBase):
    type: Literal["function"] = "function"
    function: FunctionDefinition


class UsageInfo(OpenAIBase):
    prompt_tokens: int = 0
    total_tokens: int = 0
    completion_tokens: Optional[int] = 0


class _SamplingFields(OpenAIBase):
    """Sampling fields shared by chat and completion requests."""

    model: Optional[str] = None
    frequency_penalty: Optional[float] = 0.0
    logit_bias: Optional[Dict[str, float]] = None
    max_tokens: Optional[int] = None
    n: Optional[int] = 1
    presence_penalty: Optional[float] = 0.0
    seed: Optional[int] = None
    stop: Optional[Union[str, List[str]]] = Field(default_factory=list)
    stream: Optional[bool] = False
    stream_options: Optional[StreamOptions] = None
    temperature: Optional[float] = None
    top_p: Optional[float] = None
    user: Optional[str] = None
    best_of: Optional[int] = None
    use_beam_search: bool = False
    top_k: Optional[int] = None
    min_p: Optional[float] = None
    repetition_penalty: Optional[float] = None
    length_penalty: float = 1.0
    early_stopping: bool = False
    stop_token_ids: Optional[List[int]] = Field(default_factory=list)
    include_stop_str_in_output: bool = False
    ignore_eos: bool = False
    min_tokens: int = 0
    skip_special_tokens: bool = True
    spaces_between_special_tokens: bool = True
    truncate_prompt_tokens: Optional[int] = None
    allowed_token_ids: Optional[List[int]] = None
    add_special_tokens: Optional[bool] = None
    response_format: Optional[ResponseFormat] = None
    guided_json: Optional[Union[str, Dict[str, Any]]] = None
    guided_regex: Optional[str] = None
    guided_choice: Optional[List[str]] = None
    guided_grammar: Optional[str] = None
    guided_decoding_backend: Optional[str] = None
    guided_whitespace_pattern: Optional[str] = None
    priority: int = 0

    def to_sampling_params(self, default_max_tokens: int, logprobs: Optional[int],
                           generation_defaults: Optional[Dict[str, Any]] = None) -> SamplingParams:
        gd = generation_defaults or {}
        temperature = self.temperature if self.temperature is not None else gd.get("temperature", 1.0)
        top_p = self.top_p if self.top_p is not None else gd.get("top_p", 1.0)
        top_k = self.top_k if self.top_k is not None else gd.get("top_k", -1)
        if top_k == 0:
            top_k = -1
        guided_json = self.guided_json
        if self.response_format is not None and self.response_format.type != "text":
            if self.response_format.type == "json_schema" and self.response_format.json_schema:
                js = self.response_format.json_schema
                guided_json = js.get("schema", js)
            elif guided_json is None:
                guided_json = {}
        if self.guided_grammar:
            from ...engine.grammar import validate_grammar
            validate_grammar(self.guided_grammar)      # reject unsupported grammars with a 400
        max_tokens = self.max_tokens if self.max_tokens is not None else default_max_tokens
        min_p = self.min_p if self.min_p is not None else gd.get("min_p", 0.0)
        repetition_penalty = self.repetition_penalty if self.repetition_penalty is not None \
            else gd.get("repetition_penalty", 1.0)
        if self.use_beam_search:
            # beam search ranks candidates by log-prob: deterministic, unfiltered rows (an
            # explicit non-zero temperature / top_p / top_k is a client error)
            if self.temperature not in (None, 0.0):
                raise ValueError("use_beam_search requires temperature 0")
            temperature = 0.0
            top_p = 1.0 if self.top_p is None else top_p
            top_k = -1 if self.top_k is None else top_k
            # the model's generation defaults are sampling settings: they do not apply to beams
            min_p = 0.0 if self.min_p is None else min_p
            repetition_penalty = 1.0 if self.repetition_penalty is None else repetition_penalty
            if self.stop:
                # beams end on EOS / stop_token_ids only (hypotheses are ranked on token ids)
                raise ValueError("use_beam_search does not support stop strings; "
                                 "use stop_token_ids")
        return SamplingParams(
            n=self.n or 1, best_of=self.best_of, temperature=temperature, top_p=top_p,
            top_k=top_k, min_p=min_p,
            presence_penalty=self.presence_penalty or 0.0,
            frequency_penalty=self.frequency_penalty or 0.0,
            repetition_penalty=repetition_penalty,
            seed=self.seed, stop=self.stop, stop_token_ids=self.stop_token_ids,
            ignore_eos=self.ignore_eos, max_tokens=max(1, max_tokens), min_tokens=self.min_tokens,
            logprobs=logprobs, skip_special_tokens=self.skip_special_tokens,
            spaces_between_special_tokens=self.spaces_between_special_tokens,
            include_stop_str_in_output=self.include_stop_str_in_output,
            logit_bias={int(k): float(v) for k, v in self.logit_bias.items()}
            if self.logit_bias else None,
            allowed_token_ids=self.allowed_token_ids,
            guided_choice=self.guided_choice, guided_regex=self.guided_regex,
            guided_grammar=self.guided_grammar,
            guided_json=guided_json, use_beam_search=self.use_beam_search,
            length_penalty=self.length_penalty, early_stopping=self.early_stopping)


class ChatCompletionRequest(_SamplingFields):
    messages: List[Dict[str, Any]]
    logprobs: Optional[bool] = False
    top_logprobs: Optional[int] = 0
    max_completion_tokens: Optional[int] = None
    tools: Optional[List[ChatCompletionToolsParam]] = None
    tool_choice: Optional[Union[Literal["none", "auto", "required"], Dict[str, Any]]] = "none"
    parallel_tool_calls: Optional[bool] = True
    echo: bool = False
    add_generation_prompt: bool = True
    continue_final_message: bool = False
    documents: Optional[List[Dict[str, str]]] = None
    chat_template: Optional[str] = None
    chat_template_kwargs: Optional[Dict[str, Any]] = None


class CompletionRequest(_SamplingFields):
    prompt: Union[List[int], List[List[int]], str, List[str]]
    echo: Optional[bool] = False
    logprobs: Optional[int] = None
    suffix: Optional[str] = None


class EmbeddingRequest(OpenAIBase):
    model: Optional[str] = None
    input: Union[List[int], List[List[int]], str, List[str]]
    encoding_format: Literal["float", "base64"] = "float"
    dimensions: Optional[int] = None
    user: Optional[str] = None
    additional_data: Optional[Any] = None
    truncate_prompt_tokens: Optional[int] = None


# ----------------------------------------------------------------------------- responses

class Logprob(OpenAIBase):
    token: str
    logprob: float
    bytes: Optional[List[int]] = None


class ChatLogprobContent(Logprob):
    top_logprobs: List[Logprob] = Field(default_factory=list)


class ChatLogprobs(OpenAIBase):
    content: Optional[List[ChatLogprobContent]] = None


class CompletionLogprobs(OpenAIBase):
    text_offset: List[int] = Field(default_factory=list)
    token_logprobs: List[Optional[float]] = Field(default_factory=list)
    tokens: List[str] = Field(default_factory=list)
    top_logprobs: List[Optional[Dict[str, float]]] = Field(default_factory=list)


class CompletionResponseChoice(OpenAIBase):
    index: int
    text: str
    logprobs: Optional[CompletionLogprobs] = None
    finish_reason: Optional[str] = None
    stop_reason: Optional[Union[int, str]] = None


class CompletionResponse(OpenAIBase):
    id: str = Field(default_factory=lambda: random_id("cmpl"))
    object: str = "text_completion"
    created: int = Field(default_factory=lambda: int(time.time()))
    model: str
    choices: List[CompletionResponseChoice]
    usage: UsageInfo


class CompletionStreamChoice(OpenAIBase):
    index: int
    text: str
    logprobs: Optional[CompletionLogprobs] = None
    finish_reason: Optional[str] = None
    stop_reason: Optional[Union[int, str]] = None


class CompletionStreamResponse(OpenAIBase):
    id: str
    object: str = "text_completion"
    created: int
    model: str
    choices: List[CompletionStreamChoice]
    usage: Optional[UsageInfo] = None


class FunctionCall(OpenAIBase):
    name: str
    arguments: str


class ToolCall(OpenAIBase):
    id: str = Field(default_factory=lambda: random_id("chatcmpl-tool"))
    type: Literal["function"] = "function"
    function: FunctionCall


class DeltaFunctionCall(OpenAIBase):
    name: Optional[str] = None
    arguments: Optional[str] = None


class DeltaToolCall(OpenAIBase):
    id: Optional[str] = None
    type: Optional[Literal["function"]] = None
    index: int
    function: Optional[DeltaFunctionCall] = None


class ChatMessage(OpenAIBase):
    role: str
    content: Optional[str] = None
    reasoning_content: Optional[str] = None
    tool_calls: List[ToolCall] = Field(default_factory=list)


class ChatCompletionResponseChoice(OpenAIBase):
    index: int
    message: ChatMessage
    logprobs: Optional[ChatLogprobs] = None
    finish_reason: Optional[str] = "stop"
    stop_reason: Optional[Union[int, str]] = None


class ChatCompletionResponse(OpenAIBase):
    id: str = Field(default_factory=lambda: random_id("chatcmpl"))
    object: Literal["chat.completion"] = "chat.completion"
    created: int = Field(default_factory=lambda: int(time.time()))
    model: str
    choices: List[ChatCompletionResponseChoice]
    usage: UsageInfo


class DeltaMessage(OpenAIBase):
    role: Optional[str] = None
    content: Optional[str] = None
    tool_calls: List[DeltaToolCall] = Field(default_factory=list)


class ChatCompletionResponseStreamChoice(OpenAIBase):
    index: int
    delta: DeltaMessage
    logprobs: Optional[ChatLogprobs] = None
    finish_reason: Optional[str] = None
    stop_reason: Optional[Union[int, str]] = None


class ChatCompletionStreamResponse(OpenAIBase):
    id: str
    object: Literal["chat.completion.chunk"] = "chat.completion.chunk"
    created: int
    model: str
    choices: List[ChatCompletionResponseStreamChoice]
    usage: Optional[UsageInfo] = None


class EmbeddingResponseData(OpenAIBase):
    index: int
    object: str = "embedding"
    embedding: Union[List[float], str]


class EmbeddingResponse(OpenAIBase):
    id: str = Field(default_factory=lambda: random_id("embd"))
    object: str = "list"
    created: int = Field(default_factory=lambda: int(time.time()))
    model: str
    data: List[EmbeddingResponseData]
    usage: UsageInfo


class ModelCard(OpenAIBase):
    id: str
    object: str = "model"
    created: int = Field(default_factory=lambda: int(time.time()))
    owned_by: str = "enterprise-inference-amd"
    root: Optional[str] = None
    parent: Optional[str] = None
    max_model_len: Optional[int] = None


class ModelList(OpenAIBase):
    object: str = "list"
    data: List[ModelCard] = Field(default_factory=list)
