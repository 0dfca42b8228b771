{{- define "gw.name" -}}{{ .Release.Name }}{{- end -}}
{{- define "gw.service" -}}{{ .Release.Name }}-service{{- end -}}
{{- define "gw.labels" -}}
app.kubernetes.io/name: genai-gateway
app.kubernetes.io/instance: {{ .Release.Name }}
app.kubernetes.io/managed-by: {{ .Release.Service }}
{{- end -}}
{{- define "gw.pgHost" -}}{{ .Release.Name }}-postgresql{{- end -}}
{{- define "gw.redisHost" -}}{{ .Release.Name }}-redis-master{{- end -}}
{{- define "gw.tlsSecret" -}}{{ .Values.ingress.tlsSecretName | default .Values.host }}{{- end -}}
