{{- define "tei.fullname" -}}
{{- if contains .Chart.Name .Release.Name -}}{{ .Release.Name | trunc 63 | trimSuffix "-" }}
{{- else -}}{{ printf "%s-%s" .Release.Name .Chart.Name | trunc 63 | trimSuffix "-" }}{{- end -}}
{{- end -}}
{{- define "tei.prefix" -}}
{{- $last := .Values.EMBEDDING_MODEL_ID | splitList "/" | last -}}
{{- if .Values.accelDevice -}}{{ $last }}{{- else -}}{{ $last }}-teicpu{{- end -}}
{{- end -}}
