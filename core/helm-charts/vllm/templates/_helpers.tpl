{{/* Release-derived names (a release whose name contains the chart name keeps it as is). */}}
{{- define "vllm.fullname" -}}
{{- if contains .Chart.Name .Release.Name -}}
{{- .Release.Name | trunc 63 | trimSuffix "-" -}}
{{- else -}}
{{- printf "%s-%s" .Release.Name .Chart.Name | trunc 63 | trimSuffix "-" -}}
{{- end -}}
{{- end -}}

{{- define "vllm.labels" -}}
app.kubernetes.io/name: vllm
app.kubernetes.io/instance: {{ .Release.Name }}
app.kubernetes.io/managed-by: {{ .Release.Service }}
helm.sh/chart: {{ .Chart.Name }}-{{ .Chart.Version }}
{{- end -}}

{{- define "vllm.selectorLabels" -}}
app.kubernetes.io/name: vllm
app.kubernetes.io/instance: {{ .Release.Name }}
{{- end -}}

{{/* Per-model configuration: modelConfigs[LLM_MODEL_ID] or defaultModelConfigs. */}}
{{- define "vllm.modelConfig" -}}
{{- $mc := index .Values.modelConfigs .Values.LLM_MODEL_ID | default .Values.defaultModelConfigs -}}
{{- toYaml $mc -}}
{{- end -}}

{{/* URL path prefix: last segment of the model id (+ -vllmcpu on the CPU path). */}}
{{- define "vllm.pathPrefix" -}}
{{- $last := .Values.LLM_MODEL_ID | splitList "/" | last -}}
{{- if .Values.accelDevice -}}{{ $last }}{{- else -}}{{ $last }}-vllmcpu{{- end -}}
{{- end -}}
